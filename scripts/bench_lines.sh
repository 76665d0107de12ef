#!/bin/bash
# The BASELINE config bench lines on one GPU (C2 default with CPU baseline, C3
# on one GPU, C4, C5, MCMC, MALA) plus a rocprofv3 kernel-stats pass of C4;
# each step under its own limit, stopping at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/lines
mkdir -p $O
run() {  # $1 = name, rest = bench args
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/$name.log; exit $rc; fi
  tail -1 $O/$name.log > $O/$name.json
}
run c2
run c3_64tiles --total-tiles 64 --no-cpu-baseline
run c3_9tiles --tiles-per-gpu 9 --no-cpu-baseline --no-vs-ref  # ~ a C3 rank share (64 tiles / 8 GPUs), square grid
run c4 --workload c4 --no-cpu-baseline
run c5 --workload c5 --no-cpu-baseline
run mcmc --workload mcmc
run mala --kernel mala --no-cpu-baseline
run agg --workload agg --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_c4 -o run -- \
  python3 bench.py --workload c4 --no-cpu-baseline --no-full-run > $O/prof_c4.log 2>&1
echo "prof_c4 rc=$?"
