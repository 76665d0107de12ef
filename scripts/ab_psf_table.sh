#!/bin/bash
# Radial PSF table (M71 sweeps): the parity / equality tests through it, then
# a same-box A/B of the C2 and C4 bench lines without and with it
# (SMCDET_MH_PSF_TABLE = 8192, opt-in; the default is the exp2/log2 form, with
# the 1/v cache at 32x32), alternating.  Each GPU step has its own limit; a crash or timeout
# ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/ab_tb
mkdir -p $D
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_psf_cache.py tests/test_gpu_teacher.py \
  tests/test_gpu_parity.py tests/test_gpu_fused_step.py} -v -p no:cacheprovider --timeout 200 \
  --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $D/pytest.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
Q="--no-cpu-baseline --no-full-run --no-vs-ref --no-spread --no-c3"
for rep in ${REPS:-1 2 3}; do
  for fl in 0 8192; do
    for wl in ${WLS:-c2 c4}; do
      timeout -k 10 200 python bench.py $Q --workload $wl --mh-debug-flags $fl \
        > $D/${wl}_f${fl}_r${rep}.json 2> $D/${wl}_f${fl}_r${rep}.err
      rc=$?; [ $rc -ne 0 ] && { echo "bench $wl $fl rc=$rc"; tail -5 $D/${wl}_f${fl}_r${rep}.err; exit $rc; }
      python - "$D" "$wl" "$fl" "$rep" <<'PY'
import json, sys
d = json.loads(open(f"{sys.argv[1]}/{sys.argv[2]}_f{sys.argv[3]}_r{sys.argv[4]}.json").read().strip().splitlines()[-1])
print(sys.argv[2], "flags", sys.argv[3], "rep", sys.argv[4], "value %.4g" % d["value"],
      "ms/step %.4f" % d["ms_per_step"], "mh_ms %.4f" % d["roofline"]["kernel_ms"], flush=True)
PY
    done
  done
done
if [ -n "${NEWTESTS:-}" ]; then
  SMCDET_PAIRED_OUT=$D/paired.json timeout -k 10 900 python -u -m pytest $NEWTESTS -v -s \
    -p no:cacheprovider --timeout 400 --timeout-method thread > $D/pytest_new.log 2>&1
  rc=$?; echo "new tests rc=$rc"; grep -E "^FAILED|passed|failed" $D/pytest_new.log | tail -8
fi
if [ -n "${BISECT:-}" ]; then
  timeout -k 10 600 python -u scripts/paired_bisect.py --seeds $BISECT --out $D/paired_bisect.json \
    > $D/paired_bisect.log 2>&1
  rc=$?; echo "bisect rc=$rc"; tail -40 $D/paired_bisect.log
fi
