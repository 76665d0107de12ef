#!/bin/bash
# One GPU pass of a session: the GPU suite, smoke, the default bench line, the
# driver's torchrun N=1 path (RCCL process group of one rank), and the
# rocprofv3 kernel-trace + PMC passes of the C2 MH launch summarised into
# gpurun_out/pmc_mh_r04.json (scripts/pmc_summary.py).  Each GPU step has its
# own time limit; a crash, abort or timeout ends the script (test failures,
# rc 1, do not).  STEPS="pytest smoke bench torchrun1 profile" selects steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-"pytest smoke bench torchrun1 host profile large"}
step() {
  echo "$1 rc=$2"
  if [ "$2" -ne 0 ] && [ "$2" -ne 1 ]; then echo "stopping after $1"; exit "$2"; fi
}
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has pytest; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${PYTEST_ARGS:---ignore=tests/test_gpu_large_tile.py} \
    > gpurun_out/pytest_gpu.log 2>&1
  step pytest $?
  grep -E "^FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -8
fi
if has smoke; then
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
  step smoke $?
  tail -2 gpurun_out/smoke.log
fi
if has bench; then
  timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
  step bench $?
  tail -c 600 gpurun_out/bench.log; echo
fi
if has torchrun1; then
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 > gpurun_out/bench_torchrun1.log 2>&1
  step torchrun1 $?
  tail -c 400 gpurun_out/bench_torchrun1.log; echo
fi
if has host; then  # host-side issue cost of a step vs its GPU time
  timeout -k 10 200 python scripts/host_overhead.py > gpurun_out/host_overhead.json 2>gpurun_out/host_overhead.err
  step host $?
  cat gpurun_out/host_overhead.json
fi
if has profile; then
  OUT=gpurun_out/prof SUMMARY=gpurun_out/pmc_mh_r04.json \
    SQ="SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM" \
    bash scripts/profile.sh
  step profile $?
  cat gpurun_out/prof/summary.txt | tail -20
  tr=$(find gpurun_out/prof/trace -name 'run_kernel_trace.csv' | head -1)
  if [ -n "$tr" ]; then
    python scripts/step_attribution.py "$tr" --json gpurun_out/step_attribution.json | tail -8
  fi
fi
if has large; then  # the global-memory (large-tile) paths, last
  timeout -k 10 300 python -u -m pytest tests/test_gpu_large_tile.py -v -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_large.log 2>&1
  step large $?
  grep -E "^FAILED|passed|failed" gpurun_out/pytest_large.log | tail -8
fi
