"""Per-SIMD composition of a k = 2 launch from an FC_PHASE_PROF dump (slot 0: loop cycles,
slot 20: SIMD key): usage python tools/deal_report.py FILE n_chains [groups]"""
import sys
from collections import defaultdict
import numpy as np
f, C = sys.argv[1], int(sys.argv[2])
G = int(sys.argv[3]) if len(sys.argv) > 3 else 10
raw = np.fromfile(f, dtype=np.int64).reshape(-1, C, 24)
last = raw[-1]
tot, key = last[:, 0].astype(np.float64), last[:, 20]
grp = np.arange(C) % G
print("per group mean / max Mcyc:", " ".join(f"{g}:{tot[grp == g].mean()/1e6:.1f}/{tot[grp == g].max()/1e6:.1f}" for g in range(G)))
simd = defaultdict(list)
for c in range(C):
    simd[int(key[c])].append(c)
rows = []
for k, cs in simd.items():
    rows.append((max(tot[c] for c in cs), len(cs), sorted(int(grp[c]) for c in cs)))
rows.sort(reverse=True)
print("SIMDs", len(rows), "waves/SIMD histogram", np.bincount([r[1] for r in rows]).tolist())
print("slowest SIMDs (max Mcyc, waves, groups):")
for r in rows[:12]:
    print(f"  {r[0]/1e6:7.2f} {r[1]} {r[2]}")
slow = set(range(6, 10)) if G == 10 else set()
cnt = np.bincount([sum(1 for g in r[2] if g in slow) for r in rows])
print("slow chains (groups 6-9) per SIMD histogram", cnt.tolist())
