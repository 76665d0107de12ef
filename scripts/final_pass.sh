#!/bin/bash
# Closing GPU pass of round 3 session 3: the full GPU suite (large tiles
# included), smoke, the rocprofv3 kernel trace + PMC passes of the C2 bench
# (summary copied to profiles/ so the bench's compute.executed block is
# current), the default bench line and the driver's torchrun N=1 path.  Each
# GPU step has its own limit; a crash, abort or timeout ends the script (test
# failures, rc 1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
step() {
  echo "$1 rc=$2"
  if [ "$2" -ne 0 ] && [ "$2" -ne 1 ]; then echo "stopping after $1"; exit "$2"; fi
}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
step pytest $?
grep -E "^FAILED|passed|failed" gpurun_out/final/pytest_gpu.log | tail -6
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/final/smoke.log 2>&1
step smoke $?
tail -2 gpurun_out/final/smoke.log
OUT=gpurun_out/final/prof SUMMARY=gpurun_out/final/pmc_mh_r03.json \
  SQ="SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM" \
  bash scripts/profile.sh
step profile $?
tail -12 gpurun_out/final/prof/summary.txt
cp gpurun_out/final/pmc_mh_r03.json profiles/pmc_mh_r03.json
tr=$(find gpurun_out/final/prof/trace -name 'run_kernel_trace.csv' | head -1)
[ -n "$tr" ] && python scripts/step_attribution.py "$tr" --json gpurun_out/final/step_attribution.json | tail -8
timeout -k 10 400 python bench.py > gpurun_out/final/bench.log 2>&1
step bench $?
tail -c 400 gpurun_out/final/bench.log; echo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 > gpurun_out/final/bench_torchrun1.log 2>&1
step torchrun1 $?
tail -c 300 gpurun_out/final/bench_torchrun1.log; echo
