"""Phase cycles of the k > 2 kernel (FC_PHASE_PROF build, FC_PROF_OUT dump of tools/probe_side.py)
per base group: python tools/prof_side_report.py FILE n_chains n_groups"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.int64)
C, G = int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 1
S = next(k for k in (32, 28, 24) if (raw.size // C) % k == 0)  # fc_internal.h kProfSlots
last = raw.reshape(-1, C, S)[-1].astype(np.float64)
for g in range(G):
    x = last[np.arange(C) % G == g].mean(axis=0)
    b, fl = max(x[5], 1), max(x[7], 1)
    print(f"group {g}: total {x[0] / 1e6:.2f} Mcyc  batches {x[5]:.0f}  flips {x[7]:.0f}  commit iters {x[6]:.0f}")
    print(f"  per batch: draws-gen {x[18] / b:.1f}  slots {x[17] / b:.1f}  cycles: draws {x[1] / b:.0f}  eval {x[2] / b:.0f}"
          f"  commit {x[3] / b:.0f}  book {x[4] / b:.0f}")
    print(f"  per flip: dgraph tables {x[8] / fl:.0f}  nf update {x[9] / fl:.0f}  rest-to-ent {x[10] / fl:.0f}"
          f"  commit/flip {x[3] / fl:.0f}  neighbours recounted {x[19] / fl:.2f}")
    print(f"  batch ends: stale view {x[11] / b:.3f}  entering non-hit {x[12] / b:.3f}  adj change {x[15] / b:.3f}"
          f"  slot-bound change {x[16] / b:.3f}")
    if S >= 28 and x[21] > 0:
        print(f"  multi-flip passes {x[21] / b:.2f} per batch, flips per pass {x[22] / max(x[21], 1):.2f}"
              f" ({x[22] / fl:.2f} of the flips), fallbacks {x[27] / max(x[21], 1):.2f} per pass,"
              f" one-by-one table passes {x[20] / max(x[21] - x[27], 1):.3f}")
        print(f"  multi-flip cycles per pass: members {x[23] / x[21]:.0f}  recount+entering {x[24] / x[21]:.0f}"
              f"  district tables (sequential) {x[25] / max(x[21] - x[27], 1):.0f}"
              f"  apply tail {x[26] / max(x[21] - x[27], 1):.0f}")
    if S >= 32 and x[21] > 0:
        print(f"  member selection ends per pass: cap {x[28] / x[21]:.2f}  stale view {x[29] / x[21]:.2f}"
              f"  population {x[30] / x[21]:.2f}  shared neighbour {x[31] / x[21]:.2f}")
