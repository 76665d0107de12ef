#!/bin/bash
# Closing GPU pass of a session: full GPU suite, smoke, the default bench
# line, a 2-rank gloo rehearsal of the torchrun bench, every BASELINE config's
# bench line (scripts/bench_lines.sh) and rocprofv3 kernel stats + PMC passes
# of the C2 bench (scripts/profile.sh).  Each GPU step has its own limit; a
# crash, abort or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # $1 = name, $2 = rc; test failures (1) do not stop the pass
  echo "$1 rc=$2"
  if [ "$2" -ne 0 ] && [ "$2" -ne 1 ]; then echo "stopping after $1"; exit "$2"; fi
}
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
step pytest $?
grep -E "^FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -5
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
step smoke $?
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
step bench $?
tail -1 gpurun_out/bench.log
SMCDET_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 \
  --warmup 1 --no-cpu-baseline --no-full-run --no-vs-ref > gpurun_out/bench_gloo2.log 2>&1
step bench_gloo2 $?
tail -1 gpurun_out/bench_gloo2.log
bash scripts/bench_lines.sh
step bench_lines $?
OUT=gpurun_out/prof SQ="SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM" \
  SQ2="SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
  bash scripts/profile.sh
step profile $?
