#!/bin/bash
# Tile pass (temper -> reweight -> bins): the Brent probe, the tests whose
# results go through the tile pass, the tile pass's phase cycles (trace
# build) at 512 and 256 threads, and the per-step kernel attribution of the
# C2 bench (rocprofv3 kernel trace) at both thread counts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/tile_pass
mkdir -p $D
timeout -k 10 60 ./scripts/probe/brent_probe > $D/brent_probe.txt 2>&1
rc=$?; cat $D/brent_probe.txt; [ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
TESTS=${TESTS:-"tests/test_gpu_fused_step.py tests/test_gpu_parity.py tests/test_gpu_checkpoint.py tests/test_gpu_batch.py tests/test_gpu_aggregate_large.py"}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS \
    > $D/tests.log 2>&1
  rc=$?; tail -3 $D/tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
for nt in 512 256; do
  SMCDET_TILE_THREADS=$nt SMCDET_ALLOW_STALE=1 timeout -k 10 200 python scripts/trace_phases.py 5 \
    > $D/phases_$nt.json 2> $D/phases_$nt.err
  rc=$?; echo "phases $nt rc=$rc"; [ $rc -ne 0 ] && { tail -5 $D/phases_$nt.err; exit $rc; }
  python - $D/phases_$nt.json << 'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k in ("step2", "step3", "step4"):
    print(k, {a: round(b) for a, b in d[k]["tile_cycles"].items()})
PY
done
timeout -k 10 200 python scripts/host_profile.py > $D/host_profile.txt 2>&1
rc=$?; head -30 $D/host_profile.txt; [ $rc -ne 0 ] && { echo "host_profile rc=$rc"; exit $rc; }
timeout -k 10 200 python scripts/startup_probe.py > $D/startup.log 2>&1
rc=$?; tail -1 $D/startup.log | cut -c1-600; [ $rc -ne 0 ] && { echo "startup rc=$rc"; exit $rc; }
Q="--no-cpu-baseline --no-full-run --no-vs-ref --no-spread --no-c3"
for nt in 512 256; do
  SMCDET_TILE_THREADS=$nt timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $D/trace_$nt -o run -- \
    python3 bench.py $Q --steps 20 > $D/trace_$nt.log 2>&1
  rc=$?; echo "trace $nt rc=$rc"; [ $rc -ne 0 ] && exit $rc
  tail -1 $D/trace_$nt.log | cut -c1-200
  tr=$(find $D/trace_$nt -name 'run_kernel_trace.csv' | head -1)
  python scripts/step_attribution.py "$tr" --json $D/step_attribution_$nt.json | grep -E "tile_us|sweep_us"
done
exit 0
