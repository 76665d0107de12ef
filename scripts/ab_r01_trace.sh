#!/bin/bash
# rocprofv3 kernel traces of the C2 bench for the round-1 tree (_r01) and the
# current tree on one box; per-kernel durations and the step interval.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/ab_r01_tr
mkdir -p $O
(cd _r01 && timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d $O/r01 -o run -- python3 bench.py \
  --no-cpu-baseline --no-full-run > $O/r01.log 2>&1) || { echo r01 failed; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d $O/cur -o run -- python3 bench.py \
  --no-cpu-baseline --no-full-run --no-vs-ref --no-kernel-timing > $O/cur.log 2>&1 || { echo cur failed; exit 1; }
for t in r01 cur; do
  echo "== $t"; python scripts/step_intervals.py $(find $O/$t -name "*kernel_trace.csv" | head -1) 20
done
