"""Phase cycles of the ReCom kernel (FC_PHASE_PROF build, FC_PROF_OUT dump of the last launch):
python tools/prof_recom_report.py FILE n_chains"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.int64)
C = int(sys.argv[2])
last = raw.reshape(-1, C, 32)[-1].astype(np.float64).mean(axis=0)
names = {0: "loop", 1: "edge + popM", 2: "spanning trees", 3: "  Boruvka scans", 4: "  hooks", 5: "  pointer jumps",
         6: "root choice", 7: "BFS order", 8: "subtree sums", 9: "cut choice", 10: "subset marks", 11: "step 5"}
P, T = max(last[16], 1), max(last[14], 1)
print(f"per chain: proposals {last[16]:.1f}  attempts {last[17]:.1f}  trees {last[14]:.1f}  Boruvka rounds/tree "
      f"{last[12] / T:.2f}  pointer-jump passes/tree {last[15] / T:.2f}  BFS levels/attempt {last[13] / max(last[17], 1):.1f}")
for i, nm in names.items():
    print(f"{nm:<18} {last[i] / 1e6:9.3f} Mcyc  {last[i] / last[0] * 100:5.1f} %  {last[i] / P / 1e3:9.1f} kcyc/proposal")
