#!/bin/bash
# Small-tile PSF cache: equality + 8x8 parity tests, then a same-box A/B of
# the C4 / C5 bench lines with and without the cache (SMCDET_MH_NO_PSF_CACHE),
# alternating.  Each GPU step has its own limit; a crash or timeout ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_pc; echo "A/B flag ${AB_FLAG:-2048}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_psf_cache.py tests/test_gpu_parity.py \
  tests/test_gpu_fused_step.py -v -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/ab_pc/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/ab_pc/pytest.log | tail -6
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
Q="--no-cpu-baseline --no-full-run --no-vs-ref --no-spread"
for rep in 1 2; do
  for wl in c4 c5; do
    for fl in 0 ${AB_FLAG:-2048}; do
      timeout -k 10 200 python bench.py --workload $wl $Q --mh-debug-flags $fl \
        > gpurun_out/ab_pc/${wl}_f${fl}_r${rep}.json 2> gpurun_out/ab_pc/${wl}_f${fl}_r${rep}.err
      rc=$?; [ $rc -ne 0 ] && { echo "bench $wl $fl rc=$rc"; exit $rc; }
      python - "$wl" "$fl" "$rep" <<'EOF'
import json, sys
d = json.loads(open(f"gpurun_out/ab_pc/{sys.argv[1]}_f{sys.argv[2]}_r{sys.argv[3]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], "flags", sys.argv[2], "rep", sys.argv[3], "value %.4g" % d["value"],
      "ms/step %.4f" % d["ms_per_step"], "mh_ms %.4f" % d["roofline"]["kernel_ms"])
EOF
    done
  done
done
