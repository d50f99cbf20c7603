#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of one HIP source (hipcc
-Rpass-analysis=kernel-resource-usage), for checking an instance's register budget after a
change.  Usage: python3 tools/kres.py csrc/fc_kernels.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
res = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "-o",
                      "/tmp/kres.o", src, "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:],
                     capture_output=True, text=True)
rows, cur = [], None
for line in res.stderr.splitlines():
    m = re.search(r"remark: ([^\[]+?) \[-Rpass", line)
    if not m:
        continue
    key, _, val = m.group(1).partition(":")
    key, val = key.strip(), val.strip()
    if key == "Function Name":
        cur = {"name": subprocess.run(["c++filt", val], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[key] = val
for r in rows:
    if flt in r["name"]:
        print(f'{r["name"]:<60} VGPR {r.get("VGPRs", "?"):>4} AGPR {r.get("AGPRs", "?"):>3} '
              f'vspill {r.get("VGPRs Spill", "?"):>3} sspill {r.get("SGPRs Spill", "?"):>4} '
              f'scratch {r.get("ScratchSize [bytes/lane]", "?"):>4} occ {r.get("Occupancy [waves/SIMD]", "?")}')
