#!/bin/bash
# Same-box A/B of library variants on the fixed-state MH microbench: for each
# smcdet_amd/libsmcdet_hip_<tag>.so in LIBS (plus the default build "cur"),
# interleaved REPS times, the block-form thresholds in SLOTS as variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/ab_mb_libs
mkdir -p $D
SLOTS=${SLOTS:-0,5}
V=$(echo $SLOTS | sed 's/\([-0-9]*\)/blk\1/g')
for r in $(seq 1 ${REPS:-3}); do
  for tag in cur ${LIBS:-}; do
    lib=smcdet_amd/libsmcdet_hip.so
    [ "$tag" != cur ] && lib=smcdet_amd/libsmcdet_hip_$tag.so
    out=$D/${tag}_r$r.json
    SMCDET_ALLOW_STALE=1 SMCDET_HIP_LIB=$PWD/$lib timeout -k 10 200 python scripts/mh_microbench.py \
      --persist --variants $V --block-slots $SLOTS --no-extra --rounds ${MB_ROUNDS:-7} \
      --tau ${TAU:-0.3} > $out 2>&1 || { echo "$tag rc=$?"; tail -5 $out; exit 1; }
    python3 -c "
import json; s=open('$out').read(); d=json.loads(s[s.index('{'):])['variants']
print('$tag r$r', ' '.join('%s %.4f' % (k, v['median_ms']) for k, v in d.items()))"
  done
done
