#!/bin/bash
# Same-box A/B of the C2 bench line: the round-1 tree (git worktree _r01 of
# the last round-1 commit, built in-tree) against the current tree, ROUNDS
# interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_r01
for r in $(seq 1 ${ROUNDS:-3}); do
  (cd _r01 && timeout -k 10 240 python bench.py --no-cpu-baseline --no-full-run ${BENCH_ARGS:-}) \
    > gpurun_out/ab_r01/r01_r$r.log 2>&1 || { echo "r01 failed"; tail -5 gpurun_out/ab_r01/r01_r$r.log; exit 1; }
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-full-run --no-vs-ref ${BENCH_ARGS:-} \
    > gpurun_out/ab_r01/cur_r$r.log 2>&1 || { echo "cur failed"; tail -5 gpurun_out/ab_r01/cur_r$r.log; exit 1; }
  for t in r01 cur; do
    tail -1 gpurun_out/ab_r01/${t}_r$r.log | python -c "import json,sys; d=json.load(sys.stdin); print('$t r$r', 'step_ms %.4f' % d['ms_per_step'], 'mh_ms %.4f' % d['roofline']['kernel_ms'], 'value %.4g' % d['value'])"
  done
done
