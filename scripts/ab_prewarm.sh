#!/bin/bash
# Same-box A/B of the bench's prewarm (--prewarm-s 0 vs 2), interleaved, REPS
# rounds; each line: value, ms/step, MH launch ms, and the in-run cold timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/ab_prewarm
mkdir -p $D
Q="--steps 20 --warmup 5 --no-cpu-baseline --no-vs-ref --no-full-run --no-c3 --no-legs"
for r in $(seq 1 ${REPS:-3}); do
  for pw in 0 2; do
    timeout -k 10 200 python bench.py $Q --prewarm-s $pw > $D/pw${pw}_r$r.log 2>&1 || exit $?
    python3 -c "
import json; d=json.loads(open('$D/pw${pw}_r$r.log').read().strip().splitlines()[-1])
c=(d.get('prewarm') or {}).get('cold') or {}
print('prewarm $pw rep $r value %.4g ms/step %.4f mh_ms %.4f cold_ms %s' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], c.get('ms_per_step')))"
  done
done
