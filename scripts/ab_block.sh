#!/bin/bash
# Same-box A/B of the block form of same-anchor M71 steps (default) against
# the per-pixel form (--mh-debug-flags 16384 = SMCDET_MH_NO_BLOCK): the C2
# bench step (and, with LEGS=1, the C4/C5/C3-share legs), interleaved, REPS
# rounds; then the fixed-state microbench (--persist) of the MH launch alone.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/ab_block${TAG:-}
mkdir -p $D
Q="--steps 20 --warmup 5 --no-cpu-baseline --no-vs-ref --no-full-run --no-spread"
[ "${LEGS:-0}" = "1" ] || Q="$Q --no-c3 --no-legs"
for r in $(seq 1 ${REPS:-3}); do
  for fl in 0 16384; do
    timeout -k 10 300 python bench.py $Q --mh-debug-flags $fl > $D/f${fl}_r$r.log 2>&1 || exit $?
    python3 -c "
import json; d=json.loads(open('$D/f${fl}_r$r.log').read().strip().splitlines()[-1])
legs=' '.join('%s %.4g' % (k, (d.get(k) or {}).get('value', 0)) for k in ('c4','c5','c3_rank_share','c3_strong') if d.get(k))
print('flags $fl rep $r value %.4g ms/step %.4f mh_ms %.4f %s' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], legs))"
  done
done
timeout -k 10 300 python scripts/mh_microbench.py --persist --variants blk0,blk5 --block-slots 0,5 \
  --no-extra --rounds ${MB_ROUNDS:-7} > $D/microbench.json 2>&1 || exit $?
python3 -c "
import json; s=open('$D/microbench.json').read(); d=json.loads(s[s.index('{'):])['variants']
for k,v in d.items(): print('microbench', k, 'median %.4f min %.4f ms' % (v['median_ms'], v['min_ms']))"
