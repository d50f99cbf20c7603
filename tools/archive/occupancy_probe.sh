set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp
for b in 6 9; do for C in 256 1024 2048 4096; do
echo "[b$b C$C] $(timeout -k 10 120 python3 tools/probe_c2.py $C 10000 $b 3 2>&1 | tail -1)" || exit 1
done; done
echo "[mixed C4096] $(timeout -k 10 120 python3 tools/probe_c2.py 4096 10000 -1 3 2>&1 | tail -1)"
