set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
[ "${RUN_TESTS:-1}" = 1 ] && timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo pytest rc=$?; tail -1 gpurun_out/pytest_gpu.log
for r in 1 2 3; do for tag in cur ${LIBS:-base}; do
  lib=$PWD/smcdet_amd/libsmcdet_hip.so; [ $tag != cur ] && lib=$PWD/smcdet_amd/libsmcdet_hip_$tag.so
  SMCDET_ALLOW_STALE=1 SMCDET_HIP_LIB=$lib timeout -k 10 200 python scripts/mh_microbench.py --only incremental --rounds 5 > gpurun_out/mb_$tag$r.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/mb_$tag$r.json'))['variants']; print('$tag r$r', *['%s %.1f' % (k, 1000*d[k]['median_ms']) for k in ('incremental','tile_kernel','temper_only','weights_only','resample_only')])"
done; done
