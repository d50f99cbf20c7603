#!/bin/bash
# r05b: baseline of this round's kernels -- C2 bench line, C3/C4/C5 side lines, and the C5
# contiguity-search lines: FC_FLAG_FORCE_BFS with the one-wave search and with
# the workgroup-cooperative search (tune search_waves=4), the latter under rocprofv3 --stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/r05b; mkdir -p "$OUT"
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --full-diag-steps 2 --sweep-replicas 0 > "$OUT/c2.json" 2> "$OUT/c2.err" || { echo "c2 failed"; tail -20 "$OUT/c2.err"; exit 1; }
python3 -c "import json; j=json.load(open('$OUT/c2.json')); print('c2', j['value'], j['roofline']['kernel_ms'], j['full_diagnostics']['kernel_ms'])"
for w in c3 c4 c5; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 5 --warmup 1 --chain-steps 20000 --no-cpu-baseline --full-diag-steps 0 > "$OUT/side_$w.json" 2> "$OUT/side_$w.err" || { echo "side $w failed"; tail -20 "$OUT/side_$w.err"; exit 1; }
  python3 -c "import json; j=json.load(open('$OUT/side_$w.json')); print('$w', j['value'], j['roofline']['kernel_ms'], j['config']['chains_per_gpu'])"
done
B5="bench.py --workload c5 --steps 3 --warmup 1 --chain-steps 20000 --no-cpu-baseline --full-diag-steps 0 --force-bfs"
timeout -k 10 300 python3 $B5 > "$OUT/side_c5_bfs_wave.json" 2> "$OUT/side_c5_bfs_wave.err" || { echo "c5 bfs wave failed"; tail -20 "$OUT/side_c5_bfs_wave.err"; exit 1; }
python3 -c "import json; j=json.load(open('$OUT/side_c5_bfs_wave.json')); print('c5 bfs wave', j['value'], j['roofline']['kernel_ms'], j['config']['chains_per_gpu'], j['bfs_per_proposal'], j['bfs_levels_per_search'], j['roofline']['kernel'])"
timeout -k 10 300 python3 $B5 --tune search_waves=4 > "$OUT/side_c5_bfs_coop.json" 2> "$OUT/side_c5_bfs_coop.err" || { echo "c5 bfs coop failed"; tail -20 "$OUT/side_c5_bfs_coop.err"; exit 1; }
python3 -c "import json; j=json.load(open('$OUT/side_c5_bfs_coop.json')); print('c5 bfs coop', j['value'], j['roofline']['kernel_ms'], j['config']['chains_per_gpu'], j['bfs_per_proposal'], j['bfs_levels_per_search'], j['roofline']['kernel'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c5_bfs_coop" -o run --output-format csv -- python3 $B5 --tune search_waves=4 > "$OUT/trace_c5_bfs_coop.log" 2>&1 || { echo "trace failed"; tail -20 "$OUT/trace_c5_bfs_coop.log"; exit 1; }
grep -h flip "$OUT"/trace_c5_bfs_coop/*kernel_stats.csv | head -5
echo R05B_OK
