#!/bin/bash
# AncestorBins (ABI 16) on the GPU: the tests that exercise the step's
# resampling hand-over, then a same-box A/B of the C2 bench line with the
# bins hand-over (default) and the int64 indices (--ancestor-indices),
# alternating, and the rocprofv3 kernel trace + per-step attribution of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/bins
mkdir -p $D
TESTS=${TESTS:-"tests/test_gpu_fused_step.py tests/test_gpu_parity.py tests/test_gpu_checkpoint.py tests/test_gpu_batch.py tests/test_gpu_sharded.py"}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS \
    > $D/tests.log 2>&1
  rc=$?; tail -3 $D/tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
Q="--no-cpu-baseline --no-full-run --no-vs-ref --no-spread --no-c3"
for rep in 1 2 3; do
  for v in bins indices; do
    extra=""; [ $v = indices ] && extra="--ancestor-indices"
    timeout -k 10 200 python bench.py $Q $extra > $D/c2_${v}_r$rep.json 2> $D/c2_${v}_r$rep.err
    rc=$?; [ $rc -ne 0 ] && { echo "bench $v rc=$rc"; tail -5 $D/c2_${v}_r$rep.err; exit $rc; }
    python - $D/c2_${v}_r$rep.json $v $rep << 'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "rep", sys.argv[3], "value %.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"],
      "mh_ms %.4f" % d["roofline"]["kernel_ms"], flush=True)
PY
  done
done
for v in bins indices; do
  extra=""; [ $v = indices ] && extra="--ancestor-indices"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $D/trace_$v -o run -- \
    python3 bench.py $Q $extra --steps 20 > $D/trace_$v.log 2>&1
  rc=$?; echo "trace $v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  tr=$(find $D/trace_$v -name 'run_kernel_trace.csv' | head -1)
  python scripts/step_attribution.py "$tr" --json $D/step_attribution_$v.json | grep -E "tile_us|sweep_us"
done
exit 0
