#!/bin/bash
# Launch gaps of the C2 bench step under rocprofv3 --kernel-trace: fused vs
# split step, with and without per-launch kernel timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gapb
for cfg in "fused:--fused-step" "split:" "fused_nt:--fused-step --no-kernel-timing" "split_nt:--no-kernel-timing"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/gapb/$name -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-full-run --no-vs-ref $args > gpurun_out/gapb/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/gapb/$name.log; exit 1; }
  echo "== $name $(tail -1 gpurun_out/gapb/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms %.4f" % d["ms_per_step"])')"
  python scripts/gap_summary.py $(find gpurun_out/gapb/$name -name "*kernel_trace.csv") 40 | grep -v "at::native\|rocclr" | tail -8
done
