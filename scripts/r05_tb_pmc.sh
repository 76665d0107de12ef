#!/bin/bash
# counters of the PSF-table variant (SMCDET_MH_PSF_TABLE,
# --mh-debug-flags 8192) next to the default sweep on the same box: wave
# cycles, SQ_WAIT_INST_ANY and the VALU / transcendental mix per particle-step,
# plus the MH launch durations of both (kernel trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/tb_pmc
mkdir -p $D
SQA="SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_WAVES"
SQB="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAVES"
for fl in 0 8192; do
  OUT=$D/f$fl TRACE=0 GRBM=1 SQ="$SQA" SQ2="$SQB" BENCH_ARGS="--mh-debug-flags $fl" PSTEPS=10 \
    SUMMARY=$D/f$fl.json bash scripts/profile.sh || exit $?
  echo "== flags $fl"; grep -E "SQ_|clock" $D/f$fl/summary.txt
done
