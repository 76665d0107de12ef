#!/bin/bash
# Same-box kernel A/B on identical, library-independent inputs
# (scripts/mh_microbench.py --state torch): the MH sweep of each library
# variant smcdet_amd/libsmcdet_hip_<tag>.so in LIBS plus the default build
# ("cur"), ROUNDS interleaved rounds; one summary line per (variant, round).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abk
LIBS=${LIBS:-}
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 $ROUNDS); do
  for tag in cur $LIBS; do
    lib=smcdet_amd/libsmcdet_hip.so
    [ "$tag" != cur ] && lib=smcdet_amd/libsmcdet_hip_$tag.so
    out=gpurun_out/abk/${tag}_r$r.json
    SMCDET_ALLOW_STALE=1 SMCDET_HIP_LIB=$PWD/$lib timeout -k 10 180 python scripts/mh_microbench.py \
      --only ${MB_ONLY:-incremental} --rounds 5 ${MB_ARGS:-} > $out 2> $out.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; tail -5 $out.err; exit $rc; fi
    python -c "import json; d=json.load(open('$out'))['variants']['${MB_ONLY:-incremental}']; print('$tag', 'r$r', '${MB_ONLY:-incremental}', 'median_ms %.4f' % d['median_ms'], 'min_ms %.4f' % d['min_ms'])"
  done
done
