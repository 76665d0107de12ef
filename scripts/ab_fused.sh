#!/bin/bash
# Same-box A/B of the fused SMC step (one launch: sweep + tile pass) against
# the split step (two launches), on the C2 bench; optional GPU tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -15
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
for i in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-run --fused-step ${BENCH_ARGS:-} > gpurun_out/b_fused_$i.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-run ${BENCH_ARGS:-} > gpurun_out/b_split_$i.log 2>&1 || exit $?
done
for f in gpurun_out/b_*.log; do
  python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', 'step_ms %.4f' % d['ms_per_step'], 'mh_ms %.4f' % d['roofline']['kernel_ms'])"
done
