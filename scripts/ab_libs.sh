#!/bin/bash
# Same-box A/B of library variants: for each smcdet_amd/libsmcdet_hip_<tag>.so
# named in LIBS (plus the default build, tag "cur"), run the bench workloads in
# WORKLOADS and print one summary line per (workload, variant).  Rounds are
# interleaved (ROUNDS times over all variants) so clock drift hits all alike.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
LIBS=${LIBS:-}
WORKLOADS=${WORKLOADS:-c4}
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for wl in $WORKLOADS; do
    for tag in cur $LIBS; do
      lib=smcdet_amd/libsmcdet_hip.so
      [ "$tag" != cur ] && lib=smcdet_amd/libsmcdet_hip_$tag.so
      out=gpurun_out/ab/${wl}_${tag}_r$r.json
      # variants built elsewhere (e.g. an older commit) carry another source hash
      SMCDET_ALLOW_STALE=1 SMCDET_HIP_LIB=$PWD/$lib timeout -k 10 240 python bench.py --workload $wl --no-cpu-baseline \
        --no-full-run ${BENCH_ARGS:-} > $out.log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "$wl $tag rc=$rc"; tail -5 $out.log; exit $rc; fi
      tail -1 $out.log > $out
      python -c "import json; d=json.load(open('$out')); print('$wl', '$tag', 'r$r', '%.4g' % d['value'], 'step_ms %.4f' % d['ms_per_step'], 'mh_ms', d.get('roofline', {}).get('kernel_ms'))"
    done
  done
done
