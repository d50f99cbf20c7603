set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for rep in 1 2; do
for cfg in "deal.so:" "deal.so:deal=-1"; do
  L=${cfg%%:*}; T=${cfg#*:}
  for b in -1 9; do
    echo "[$L tune=$T] $(FC_TUNE=$T FC_LIB_PATH=$PWD/ablibs/$L timeout -k 10 120 python3 tools/probe_c2.py 4096 100000 $b 3 2>&1 | tail -1)" || exit 1
  done
done
done
