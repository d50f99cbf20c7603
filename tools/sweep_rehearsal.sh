#!/bin/bash
# The sweep runner over two ranks on one GPU (gloo, both ranks on device 0) against one rank:
# every output file identical (the sweep summaries' timing fields aside).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
S=/tmp/sweep_reh; rm -rf $S; mkdir -p $S
ARGS="--replicas 3 --steps ${STEPS:-5000}"
timeout -k 10 300 python3 -m flipcomplexityempirical_amd.sweep $S/n1 $ARGS > $S/n1.log 2>&1 || { echo "n1 failed"; tail -20 $S/n1.log; exit 1; }
FC_BENCH_BACKEND=gloo FC_BENCH_DEVICE=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 -m flipcomplexityempirical_amd.sweep $S/n2 $ARGS > $S/n2.log 2>&1 || { echo "n2 failed"; tail -20 $S/n2.log; exit 1; }
python3 - "$S" <<'PY'
import hashlib, json, os, sys
S = sys.argv[1]
def tree(d):
    out = {}
    for dp, _, fs in os.walk(d):
        for f in fs:
            p = os.path.join(dp, f)
            rel = os.path.relpath(p, d)
            if rel.endswith(".json"):
                j = json.load(open(p)); j.pop("timing", None); j.pop("ranks", None)
                out[rel] = hashlib.md5(json.dumps(j, sort_keys=True).encode()).hexdigest()
            else:
                out[rel] = hashlib.md5(open(p, "rb").read()).hexdigest()
    return out
a, b = tree(S + "/n1"), tree(S + "/n2")
diff = sorted(k for k in set(a) | set(b) if a.get(k) != b.get(k))
print(json.dumps({"files_one_rank": len(a), "files_two_ranks": len(b), "differing": diff[:20], "identical": not diff}))
sys.exit(1 if diff else 0)
PY
