set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/blk${TAG:-}
mkdir -p $D
if [ "${TESTS:-1}" = "1" ]; then
timeout -k 10 600 python -u -m pytest ${TESTFILES:-tests/test_gpu_psf_cache.py} -v -p no:cacheprovider --timeout 240 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $D/pytest.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for tau in ${TAUS:-0.3}; do
timeout -k 10 400 python scripts/mh_microbench.py --persist --variants ${VARIANTS:-blk0,blk5,blk-5} \
  --block-slots 0,5,-5 --no-extra --rounds ${MB_ROUNDS:-9} --tau $tau > $D/mb_tau$tau.json 2>&1 || exit $?
python3 -c "
import json; s=open('$D/mb_tau$tau.json').read(); d=json.loads(s[s.index('{'):])['variants']
for k,v in d.items(): print('tau $tau', k, 'median %.4f min %.4f ms' % (v['median_ms'], v['min_ms']))"
done
if [ "${AB:-0}" = "1" ]; then REPS=${REPS:-3} LEGS=${LEGS:-0} TAG=${TAG:-} bash scripts/ab_block.sh || exit $?; fi
