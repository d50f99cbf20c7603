"""Summarise FC_PROF_OUT dumps of the FC_PHASE_PROF build: per base group (chain % groups),
mean per-chain s_memtime cycles per phase of the last launch, per batch and per applied flip.
usage: python tools/prof_report.py FILE n_chains [groups]"""
import sys
import numpy as np
f, C = sys.argv[1], int(sys.argv[2])
G = int(sys.argv[3]) if len(sys.argv) > 3 else 10
raw = np.fromfile(f, dtype=np.int64)
S = next(k for k in (32, 28, 24, 16, 8) if (raw.size // C) % k == 0)
rec = raw.reshape(-1, C, S)
last = rec[-1].astype(np.float64)
names = ["total", "draws", "eval", "commit", "book", "batches", "commit_it", "applied"]
print("grp  total_Mcyc  batches  applied  commit_it | per batch: draws  eval  commit  book | commit/applied")
for g in range(G):
    x = last[np.arange(C) % G == g].mean(axis=0)
    b = max(x[5], 1)
    print(f"{g:3d}  {x[0]/1e6:9.2f}  {x[5]:8.0f} {x[7]:8.0f} {x[6]:9.0f} | {x[1]/b:8.0f} {x[2]/b:5.0f} {x[3]/b:7.0f} {x[4]/b:5.0f} | {x[3]/max(x[7],1):8.0f}")
if S >= 16:
    print("grp | per iteration: verdict | one-event classify/apply per one-event flip | per segment, segments/batch | share: verdict one-event segment other")
    for g in range(G):
        x = last[np.arange(C) % G == g].mean(axis=0)
        it = max(x[6], 1)
        ncm = max(x[3], 1)
        oe = max(x[7] - 0, 1)
        print(f"{g:3d} | {x[8]/it:8.0f} | {x[9]/oe:8.0f} {x[10]/oe:8.0f} | {x[11]/max(x[12],1):8.0f} {x[12]/max(x[5],1):6.2f}"
              f" | {x[8]/ncm:5.2f} {(x[9]+x[10])/ncm:5.2f} {x[11]/ncm:5.2f} {1-(x[8]+x[9]+x[10]+x[11])/ncm:5.2f}")
if S >= 16:
    print("grp | per batch: stale-view cut  entering-non-hit cut  all slots committed")
    for g in range(G):
        x = last[np.arange(C) % G == g].mean(axis=0)
        b = max(x[5], 1)
        print(f"{g:3d} | {x[13]/b:6.3f} {x[14]/b:6.3f} {x[15]/b:6.3f}")
if S >= 24:
    print("grp | reeval: cycles per call, calls per batch | segment: marks, marks+conflicts+entering per segment, mark rounds")
    for g in range(G):
        x = last[np.arange(C) % G == g].mean(axis=0)
        b = max(x[5], 1)
        print(f"{g:3d} | {x[16]/max(x[17],1):8.0f} {x[17]/b:6.2f} | {x[18]/max(x[12],1):8.0f} {x[19]/max(x[12],1):8.0f} {x[21]/max(x[12],1):6.2f}")
if S >= 28:
    print("grp | per batch: slots (proposal candidates), band rebuilds, cycles per rebuild")
    for g in range(G):
        x = last[np.arange(C) % G == g].mean(axis=0)
        b = max(x[5], 1)
        print(f"{g:3d} | {x[24]/b:6.2f} {x[22]/b:6.3f} {x[23]/max(x[22],1):8.0f}")
if S >= 32:
    print("grp | per batch: commit set-up, last no-event iteration, after a segment pass (incl. reeval), after a one-event apply (incl. reeval) | commit left")
    for g in range(G):
        x = last[np.arange(C) % G == g].mean(axis=0)
        b = max(x[5], 1)
        known = x[8] + x[9] + x[10] + x[11] + x[25] + x[27] + x[29] + x[30]
        print(f"{g:3d} | {x[27]/b:8.0f} {x[25]/b:8.0f} {x[29]/b:8.0f} {x[30]/b:8.0f} | {(x[3]-known)/b:8.0f}")
print("max chain total Mcyc", last[:, 0].max() / 1e6, "argmax", int(last[:, 0].argmax()))
tot = last[:, 0]
print("per group total Mcyc mean / p90 / max:",
      " ".join(f"{g}:{tot[np.arange(C) % G == g].mean()/1e6:.1f}/{np.percentile(tot[np.arange(C) % G == g], 90)/1e6:.1f}/{tot[np.arange(C) % G == g].max()/1e6:.1f}" for g in range(G)))
