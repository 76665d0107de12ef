#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats, and
# (optionally) the ISA issue-cost probe and the MH microbench.  Every GPU step
# has its own limit; a crash/timeout/abort ends the script (test failures do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
stop_on_crash() {  # $1 = rc, $2 = step
  echo "$2 rc=$1"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi
}
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu ${PYTEST_X--x} -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  stop_on_crash $? pytest
  grep -E "^FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -15
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
  stop_on_crash $? smoke
  tail -2 gpurun_out/smoke.log
fi
if [ "${RUN_BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  stop_on_crash $? bench
  tail -1 gpurun_out/bench.log
fi
if [ "${RUN_PROF:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  stop_on_crash $? rocprof
  tail -1 gpurun_out/prof.log
fi
if [ "${RUN_PROBE:-0}" = "1" ]; then
  timeout -k 10 60 ./scripts/probe/isa_probe > gpurun_out/probe.log 2>&1
  stop_on_crash $? probe
  cat gpurun_out/probe.log
fi
if [ "${RUN_MICRO:-0}" = "1" ]; then
  timeout -k 10 300 python scripts/mh_microbench.py ${MICRO_ARGS:-} > gpurun_out/micro.log 2>&1
  stop_on_crash $? micro
  cat gpurun_out/micro.log
fi
