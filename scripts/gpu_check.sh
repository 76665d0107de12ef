#!/bin/bash
# GPU-box check: parity tests, smoke, short bench.  Every GPU step has its own
# time limit; a crash/timeout/abort ends the script (test failures do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok_or_stop() {  # $1 = rc, $2 = step
  local rc=$1
  echo "$2 rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $2"; exit "$rc"; fi
}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider \
  ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
ok_or_stop $? pytest
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
ok_or_stop $? smoke
tail -3 gpurun_out/smoke.log
if [ "${RUN_BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/bench.log 2>&1
  ok_or_stop $? bench
  tail -2 gpurun_out/bench.log
fi
