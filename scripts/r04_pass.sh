#!/bin/bash
# Round-4 GPU pass: selected tests, the bench line, the rocprofv3 kernel trace
# + PMC passes of the C2 MH launch at HEAD (summary -> gpurun_out/r04/
# pmc_mh_r04.json), and a PMC pass of the opt-in PSF-table sweep (LDS
# instructions and bank conflicts, the A/B's cause).  Each GPU step has its
# own limit; a crash, abort or timeout ends the script (test failures, rc 1,
# do not).  STEPS selects: tests bench profile tbpmc postbench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/r04
mkdir -p $D
STEPS=${STEPS:-"tests bench profile tbpmc"}
has() { [[ " $STEPS " == *" $1 "* ]]; }
step() {
  echo "$1 rc=$2"
  if [ "$2" -ne 0 ] && [ "$2" -ne 1 ]; then echo "stopping after $1"; exit "$2"; fi
}
SQSET="SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM"
if has tests; then
  SMCDET_PAIRED_OUT=$D/paired.json timeout -k 10 900 python -u -m pytest ${TESTS:-tests -m gpu} -v \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
  step tests $?
  grep -E "^FAILED|passed|failed" $D/pytest.log | tail -12
fi
if has bench; then
  timeout -k 10 400 python bench.py > $D/bench.log 2>&1
  step bench $?
  tail -c 700 $D/bench.log; echo
fi
if has profile; then
  OUT=$D/prof SUMMARY=$D/pmc_mh_r04.json SQ="$SQSET" SQ2="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
    bash scripts/profile.sh
  step profile $?
  tail -20 $D/prof/summary.txt
  tr=$(find $D/prof/trace -name 'run_kernel_trace.csv' | head -1)
  [ -n "$tr" ] && python scripts/step_attribution.py "$tr" --json $D/step_attribution.json | tail -8
fi
if has tbpmc; then
  OUT=$D/prof_tb TRACE=0 GRBM=0 BENCH_ARGS="--mh-debug-flags 8192" \
    SQ="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32" \
    SUMMARY=$D/pmc_mh_tb.json bash scripts/profile.sh
  step tbpmc $?
  tail -12 $D/prof_tb/summary.txt
fi
if has postbench; then
  # the bench line with this pass's counters: the PMC summary (same library
  # source hash) goes where bench.py reads it, then the default bench runs
  cp $D/pmc_mh_r04.json profiles/pmc_mh_r04.json
  timeout -k 10 400 python bench.py > $D/bench_post.log 2>&1
  step postbench $?
  tail -c 400 $D/bench_post.log; echo
fi
