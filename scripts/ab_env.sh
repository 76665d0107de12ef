#!/bin/bash
# Same-box A/B of an environment switch: bench WORKLOADS with ENVVAR unset and
# set to 1, interleaved over ROUNDS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abenv
WORKLOADS=${WORKLOADS:-c2}
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 $ROUNDS); do
  for wl in $WORKLOADS; do
    for v in 0 1; do
      out=gpurun_out/abenv/${wl}_${v}_r$r.json
      env ${ENVVAR}=$v timeout -k 10 240 python bench.py --workload $wl --no-cpu-baseline \
        --no-full-run ${BENCH_ARGS:-} > $out.log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "$wl $v rc=$rc"; tail -5 $out.log; exit $rc; fi
      tail -1 $out.log > $out
      python -c "import json; d=json.load(open('$out')); print('$wl', '$ENVVAR=$v', 'r$r', '%.4g' % d['value'], 'step_ms %.4f' % d['ms_per_step'], 'mh_ms', d.get('roofline', {}).get('kernel_ms'))"
    done
  done
done
