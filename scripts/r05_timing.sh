#!/bin/bash
# Round-5 timing check: three bench reps with the prewarm,
# then one rocprofv3 kernel trace of a bench whose trace ends with the timed
# region, and the trace's per-step attribution of its last 20 steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/r05_timing${TAG:-}
mkdir -p $D
Q="--no-cpu-baseline --no-vs-ref --no-full-run"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $Q > $D/bench_rep$r.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('$D/bench_rep$r.log').read().strip().splitlines()[-1]); print('rep $r', d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d['step_spread']['repeat_passes_ms_per_step'], d.get('prewarm',{}) and d['prewarm']['steps'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $D/trace -o run -- python3 bench.py --steps 20 --warmup 5 $Q --no-c3 --no-legs --no-spread --no-kernel-timing > $D/bench_traced.log 2>&1 || exit $?
tr=$(find $D/trace -name 'run_kernel_trace.csv' | head -1)
python3 scripts/step_attribution.py "$tr" --tail 20 --json $D/step_attribution.json
python3 -c "import json; d=json.loads(open('$D/bench_traced.log').read().strip().splitlines()[-1]); print('traced bench ms_per_step', d['ms_per_step'])"
