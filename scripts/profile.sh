#!/bin/bash
# rocprofv3 kernel trace + stats of the bench, then separate PMC passes for the
# MH kernel (counter passes never combined with other trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
KRE=${KRE:-mh_sweep}  # kernel-name regex of the PMC passes
mkdir -p $OUT
B="bench.py --steps ${PSTEPS:-20} --warmup 3 --no-cpu-baseline --no-full-run --no-vs-ref --no-c3 --no-legs --no-spread --prewarm-s 0 ${BENCH_ARGS:-}"
run() {  # $1 = name, rest = rocprofv3 args
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -T -f csv -d $OUT/$name -o run -- python3 $B > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ "${LIST:-0}" = "1" ]; then
  timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
fi
if [ "${TRACE:-1}" = "1" ]; then
  run trace --kernel-trace --stats
  run fetch --pmc FETCH_SIZE --kernel-include-regex $KRE
  run write --pmc WRITE_SIZE --kernel-include-regex $KRE
fi
if [ -n "${SQ:-}" ]; then run sq --pmc $SQ --kernel-include-regex $KRE; fi
if [ -n "${SQ2:-}" ]; then run sq2 --pmc $SQ2 --kernel-include-regex $KRE; fi
if [ -n "${SQ3:-}" ]; then run sq3 --pmc $SQ3 --kernel-include-regex $KRE; fi
# effective clock: GRBM_GUI_ACTIVE with the same pass's kernel trace (durations)
if [ "${GRBM:-1}" = "1" ]; then run grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --kernel-include-regex $KRE; fi
if [ -n "${SUMMARY:-}" ]; then
  python3 scripts/pmc_summary.py --root $OUT --json "$SUMMARY" > $OUT/summary.txt 2>&1
  echo "summary rc=$?"
fi
