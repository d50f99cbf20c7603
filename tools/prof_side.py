"""Phase cycles of a side-config run (FC_PHASE_PROF build): python tools/prof_side.py FILE n_chains"""
import sys
import numpy as np
raw = np.fromfile(sys.argv[1], dtype=np.int64)
C = int(sys.argv[2])
last = raw.reshape(-1, C, 16)[-1].astype(np.float64).mean(axis=0)
b = max(last[5], 1)
print(f"per chain: total {last[0]/1e6:.2f} Mcyc, batches {last[5]:.0f}, applied {last[7]:.0f}, commit_it {last[6]:.0f}")
print(f"per batch: draws {last[1]/b:.0f} eval {last[2]/b:.0f} commit {last[3]/b:.0f} book {last[4]/b:.0f}")
print(f"bfs: calls {last[14]:.1f}  cycles/call {last[13]/max(last[14],1):.0f}  share of total {last[13]/max(last[0],1):.3f}"
      f"  expansion share of bfs {last[15]/max(last[13],1):.3f}")
if last[11] > 0:
    n = last[11]
    print(f"per node expansion (lane-cycles): load lab/cm/record {last[8]/n:.0f}  ring reads + claims {last[9]/n:.0f}"
          f"  writes + label reads {last[10]/n:.0f}  (nodes {n:.0f})")
