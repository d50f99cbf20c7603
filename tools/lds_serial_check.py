"""Static check of a gfx950 kernel's assembly (hipcc -S -gline-tables-only) for LDS / scalar
loads that are waited on within four instructions of their issue -- reads issued one round
trip at a time (round 4 found the k = 2 kernel's ring-district reads and the k > 2 kernel's
ring reads serialized this way).  Prints (source line, count) pairs, the line
being the outermost call site in the kernel's own file.

    python tools/lds_serial_check.py kernel.s FILE_STEM [FILE_STEM ...]
"""
import collections
import re
import sys


def main(path, stems):
    pat = re.compile(r"(?:%s)\.hip:(\d+):\d+" % "|".join(map(re.escape, stems)))
    cur, seq = None, []
    for line in open(path):
        m = re.match(r"\s+\.loc\s+(\d+)\s+(\d+)", line)
        if m:
            ctx = pat.findall(line)
            f, ln = int(m.group(1)), int(m.group(2))
            cur = int(ctx[-1]) if len(ctx) > 1 else (ln if f == 0 else (int(ctx[0]) if ctx else cur))
            continue
        if re.match(r"\s+(s_|v_|ds_|global_|buffer_)", line):
            seq.append((cur, line.strip()))
    out, pending = collections.Counter(), []
    for i, (ln, ins) in enumerate(seq):
        if ins.startswith(("ds_", "s_load", "s_buffer_load")):
            pending.append((i, ln))
        m = re.match(r"s_waitcnt.*lgkmcnt\((\d+)\)", ins)
        if m:
            n = int(m.group(1))
            while len(pending) > n:
                j, l2 = pending.pop(0)
                if i - j <= 4:
                    out[l2] += 1
    for ln, c in sorted(out.items(), key=lambda t: (t[0] is None, t[0] or 0)):
        print(ln, c)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:] or ["fc_flip2", "fc_kernels"])
