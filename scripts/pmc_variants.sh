#!/bin/bash
# SQ counters of the MH kernel under each microbench variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcv
mkdir -p $OUT
SQ="SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU"
SQ2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
for v in ${VARIANTS:-incremental no_both no_likelihood no_proposal}; do
  for set in 1 2; do
    if [ $set = 1 ]; then C=$SQ; else C=$SQ2; fi
    timeout -k 10 200 rocprofv3 --pmc $C --kernel-include-regex mh_sweep -T -f csv -d $OUT/$v.$set -o run -- python3 scripts/mh_microbench.py --only $v --rounds 3 > $OUT/$v.$set.log 2>&1
    rc=$?; echo "$v.$set rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
