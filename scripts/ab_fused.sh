set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -15
if [ $rc -gt 1 ]; then exit $rc; fi
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-run > gpurun_out/b_fused_$i.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-run --split-step > gpurun_out/b_split_$i.log 2>&1 || exit $?
done
for f in gpurun_out/b_*.log; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['roofline']['kernel_ms'])"; done
