#!/bin/bash
# 1/v cache (M71 register-render tiles): equality + parity tests, then a
# same-box A/B of the C2 and C3 bench lines with and without it
# (SMCDET_MH_NO_RCP_CACHE = 4096), alternating.  Each GPU step has its own
# limit; a crash or timeout ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_rv
timeout -k 10 500 python -u -m pytest tests/test_gpu_psf_cache.py tests/test_gpu_teacher.py \
  tests/test_gpu_parity.py tests/test_gpu_fused_step.py -v -p no:cacheprovider --timeout 200 \
  --timeout-method thread > gpurun_out/ab_rv/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/ab_rv/pytest.log | tail -6
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
Q="--no-cpu-baseline --no-full-run --no-vs-ref --no-spread --no-c3"
for rep in 1 2 3; do
  for fl in 0 4096; do
    for wl in c2 c3; do
      extra=""; [ $wl = c3 ] && extra="--total-tiles 64 --steps 10 --warmup 2"
      timeout -k 10 200 python bench.py $Q $extra --mh-debug-flags $fl \
        > gpurun_out/ab_rv/${wl}_f${fl}_r${rep}.json 2> gpurun_out/ab_rv/${wl}_f${fl}_r${rep}.err
      rc=$?; [ $rc -ne 0 ] && { echo "bench $wl $fl rc=$rc"; exit $rc; }
      python - "$wl" "$fl" "$rep" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_rv/{sys.argv[1]}_f{sys.argv[2]}_r{sys.argv[3]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], "flags", sys.argv[2], "rep", sys.argv[3], "value %.4g" % d["value"],
      "ms/step %.4f" % d["ms_per_step"], "mh_ms %.4f" % d["roofline"]["kernel_ms"])
PY
    done
  done
done
