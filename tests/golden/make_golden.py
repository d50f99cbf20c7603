"""Generate tests/golden/reference_artifacts.npz from the reference's own output artifacts.

Run HERE (the container with /root/reference); the GPU box only reads the committed .npz.
Nothing from the reference is copied: the fixture holds decoded data only.

* ``*end2.png`` (``grid_chain_sec11.py:440-450`` / ``Frankenstein_chain.py:468-478``):
  ``imshow`` of the final ±1 assignment with the jet colormap -> decoded per cell
  (image row = n[0], column = n[1] (+19 for FRANK)); corner cells of sec11 are 0.
* ``*wait.txt`` (``grid_chain_sec11.py:410-411``): ``sum(waits)`` over the 100,000 yields.

Configuration keys follow the reference's file names ``{alignment}B{int(100*base)}P{int(100*pop)}``.
"""
import os
import re
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_artifacts.npz")


def decode_end2(path, nrows, ncols):
    from PIL import Image
    im = np.asarray(Image.open(path).convert("RGB")).astype(int)
    R, G, B = im[..., 0], im[..., 1], im[..., 2]
    dark = ((R > 100) & (G < 40) & (B < 40)) | ((B > 100) & (R < 40) & (G < 40))
    xs = np.where(dark.sum(0) > 0)[0]
    x0 = xs[0]
    x1 = x0
    for x in xs[1:]:
        if x != x1 + 1:
            break
        x1 = x
    ys = np.where(dark[:, x0:x1 + 1].sum(1) > 0)[0]
    y0, y1 = ys[0], ys[-1]
    cw = (x1 - x0 + 1) / ncols
    ch = (y1 - y0 + 1) / nrows
    out = np.zeros((nrows, ncols), dtype=np.int8)
    for i in range(nrows):
        for j in range(ncols):
            px = im[int(y0 + (i + 0.5) * ch), int(x0 + (j + 0.5) * cw)]
            r, g, b = px
            if r > g and r > b:
                out[i, j] = 1
            elif b > r and b > g:
                out[i, j] = -1
            else:
                out[i, j] = 0
    return out


def collect(folder, nrows, ncols):
    keys, ends, waits = [], [], []
    names = sorted(os.listdir(folder))
    for f in names:
        m = re.match(r"^(\d)B(\d+)P(\d+)end2\.png$", f)
        if not m:
            continue
        key = f[:-len("end2.png")]
        wf = os.path.join(folder, key + "wait.txt")
        if not os.path.exists(wf):
            continue
        keys.append(key)
        ends.append(decode_end2(os.path.join(folder, f), nrows, ncols))
        waits.append(int(open(wf).read().strip()))
    return np.asarray(keys), np.stack(ends), np.asarray(waits, dtype=np.int64)


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not mounted; the committed fixture is authoritative")
    s_keys, s_end, s_wait = collect(os.path.join(REF, "New_plots", "sec11"), 40, 40)
    f_keys, f_end, f_wait = collect(os.path.join(REF, "plots", "FRANK"), 20, 40)
    np.savez_compressed(OUT, sec11_keys=s_keys, sec11_end=s_end, sec11_wait=s_wait,
                        frank_keys=f_keys, frank_end=f_end, frank_wait=f_wait)
    print(f"wrote {OUT}: sec11 {len(s_keys)} configs, FRANK {len(f_keys)} configs")


if __name__ == "__main__":
    main()
