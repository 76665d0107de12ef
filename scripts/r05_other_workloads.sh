#!/bin/bash
# The README's secondary workloads re-measured at HEAD's library: MALA at the
# C2 geometry, the MHsampler cutouts and the Aggregate levels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/other_wl
mkdir -p $D
Q="--no-cpu-baseline --no-full-run --no-vs-ref --no-legs --no-c3 --no-spread"
timeout -k 10 300 python bench.py --kernel mala $Q > $D/mala.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload mcmc $Q > $D/mcmc.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload agg $Q > $D/agg.log 2>&1 || exit $?
for w in mala mcmc agg; do
  python3 -c "
import json; d=[json.loads(l) for l in open('$D/$w.log') if l.startswith('{\"metric\"')][-1]
print('$w', d['metric'], '%.4g' % d['value'], d['unit'], 'ms/step %.4f' % d['ms_per_step'])"
done
