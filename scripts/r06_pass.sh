#!/bin/bash
# Round-6 GPU pass.  STEPS selects: tests smoke probe bench profile c4pmc c5pmc postbench
# Each GPU step has its own limit; a crash, abort or timeout ends the script
# (test failures, rc 1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/r06${TAG:-}
mkdir -p $D
STEPS=${STEPS:-"tests bench"}
has() { [[ " $STEPS " == *" $1 "* ]]; }
step() {
  echo "$1 rc=$2"
  if [ "$2" -ne 0 ] && [ "$2" -ne 1 ]; then echo "stopping after $1"; exit "$2"; fi
}
SQSET="SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM"
SQ2SET="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
SQ3SET="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SCRATCH SQ_WAVES"
if has tests; then
  SMCDET_PAIRED_OUT=$D/paired.json SMCDET_PAIRED_C5_OUT=$D/paired_c5.json SMCDET_C5_STATS_OUT=$D/c5_stats.json \
    timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest ${TESTS:-tests -m gpu} -v \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
  step tests $?
  grep -E "^FAILED|passed|failed" $D/pytest.log | tail -12
fi
if has smoke; then
  timeout -k 10 240 python __graft_entry__.py smoke > $D/smoke.log 2>&1
  step smoke $?
  tail -2 $D/smoke.log
fi
if has probe; then
  [ -x scripts/probe/issue_probe ] || /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 \
    -o scripts/probe/issue_probe scripts/probe/issue_probe.hip
  timeout -k 10 120 ./scripts/probe/issue_probe > $D/issue_probe.txt 2>&1
  step probe $?
  cat $D/issue_probe.txt
fi
if has law; then
  # north_star's "log Z and ESS within 1%" by sample size (scripts/c2_law.py)
  timeout -k 10 600 python -u scripts/c2_law.py ${LAW_RUNS:-8192} > $D/c2_law.json 2> $D/c2_law.err
  step law $?
  python -c "import json; d=json.load(open('$D/c2_law.json')); print({n: {k: (round(d[n][k]['rel_diff'], 5), [round(x, 5) for x in d[n][k]['rel_diff_95']]) for k in ('logZ', 'final_ess', 'iters')} for n in ('vs_oracle', 'vs_reference')})"
fi
if has paired; then
  # every oracle run of the C2 target replayed on the GPU (tests/test_gpu_paired.py);
  # -s: every seed's line reaches the log as it is written
  SMCDET_PAIRED_ALL=1 SMCDET_PAIRED_NO_TWIN=${NO_TWIN:-1} SMCDET_PAIRED_CHUNKS=${CHUNKS:-48} \
    SMCDET_PAIRED_PART=${PART:-} \
    SMCDET_PAIRED_OUT=$D/paired_all.json timeout -k 10 ${PAIRED_LIMIT:-3000} \
    python -u -m pytest tests/test_gpu_paired.py -s -q -p no:cacheprovider --timeout 600 \
    --timeout-method thread > $D/paired_all.log 2>&1
  step paired $?
  tail -4 $D/paired_all.log
fi
if has bench; then
  timeout -k 10 400 python bench.py > $D/bench.log 2>&1
  step bench $?
  tail -c 700 $D/bench.log; echo
fi
if has profile; then
  OUT=$D/prof SUMMARY=$D/pmc_mh_r06.json SQ="$SQSET" SQ2="$SQ2SET" SQ3="$SQ3SET" \
    bash scripts/profile.sh
  step profile $?
  tail -20 $D/prof/summary.txt
  tr=$(find $D/prof/trace -name 'run_kernel_trace.csv' | head -1)
  [ -n "$tr" ] && python scripts/step_attribution.py "$tr" --json $D/step_attribution.json | tail -8
fi
if has trace; then
  # the bench line's own command (prewarm on) under a kernel trace: the last
  # 20 steps' launches are the timed steps' identical replay, whose sweep /
  # tile durations the line reports as step_attribution -- the two must agree
  mkdir -p $D/trace_bench
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $D/trace_bench -o run -- \
    python3 bench.py --no-c3 --no-legs --no-vs-ref --no-full-run --no-cpu-baseline --no-spread \
    > $D/trace_bench.log 2>&1
  step trace $?
  tr=$(find $D/trace_bench -name 'run_kernel_trace.csv' | head -1)
  [ -n "$tr" ] && python scripts/step_attribution.py "$tr" --tail 20 --json $D/trace_bench_attribution.json | tail -12
  grep '^{' $D/trace_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench line:', json.dumps({k: d['step_attribution'][k] for k in ('sweep_ms', 'tile_pass_ms', 'timed_ms_per_step')}))"
fi
if has c4pmc; then
  OUT=$D/prof_c4 BENCH_ARGS="--workload c4" SQ="$SQSET" SQ2="$SQ2SET" SQ3="$SQ3SET" \
    PSTEPS=10 bash scripts/profile.sh
  step c4pmc $?
  python3 scripts/pmc_summary.py --root $D/prof_c4 --steps-per-launch 17203200 \
    --note "rocprofv3 passes of scripts/profile.sh over bench.py --workload c4 (42 8x8 cutouts, N=4096, K=100)" \
    --json $D/pmc_mh_c4_r06.json > $D/prof_c4/summary.txt 2>&1
  tail -20 $D/prof_c4/summary.txt
fi
if has c5pmc; then
  # particle-steps per launch: 42 cutouts x 6 strata with s >= 1 x 8192 x 100
  OUT=$D/prof_c5 BENCH_ARGS="--workload c5" SQ="$SQSET" SQ2="$SQ2SET" \
    PSTEPS=10 bash scripts/profile.sh
  step c5pmc $?
  python3 scripts/pmc_summary.py --root $D/prof_c5 --steps-per-launch 206438400 \
    --note "rocprofv3 passes of scripts/profile.sh over bench.py --workload c5 (42 8x8 cutouts x 7 strata, N=8192, K=100)" \
    --json $D/pmc_mh_c5_r06.json > $D/prof_c5/summary.txt 2>&1
  tail -20 $D/prof_c5/summary.txt
fi
if has postbench; then
  for f in pmc_mh_r06.json pmc_mh_c4_r06.json pmc_mh_c5_r06.json; do
    [ -f $D/$f ] && cp $D/$f profiles/$f
  done
  timeout -k 10 400 python bench.py > $D/bench_post.log 2>&1
  step postbench $?
  tail -c 400 $D/bench_post.log; echo
fi
