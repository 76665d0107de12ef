#!/bin/bash
# CPU-only oracle statistics runs on a GPU box's host cores (no GPU use):
# float64 and float32-class C2 runs of the same seeds in two processes, each
# stopping at its own time limit (every run is written as it completes).
#   FIRST=<first seed> N=<runs> LIMIT=<seconds> bash scripts/oracle_box.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/oracle_box${TAG:-}
mkdir -p $D
export OMP_WAIT_POLICY=passive
mkdir -p $D/a $D/b   # one output directory per process (no read-modify-write race)
FIRST=${FIRST:-1000}; N=${N:-200}; LIMIT=${LIMIT:-1080}
W=${WHAT:-c2_moderate_4096_k100}
SMCDET_ORACLE_OUT=$D/a timeout -k 10 $LIMIT python -u tests/golden/make_oracle_stats.py $W $N $FIRST 8 f64 > $D/f64.log 2>&1 &
p1=$!
if [ "$W" = "c5" ]; then
  SMCDET_ORACLE_OUT=$D/b timeout -k 10 $LIMIT python -u tests/golden/make_oracle_stats.py c5 $N $((FIRST + 500)) 8 f64 > $D/f64b.log 2>&1 &
elif [ -n "${F64B:-}" ]; then
  SMCDET_ORACLE_OUT=$D/b timeout -k 10 $LIMIT python -u tests/golden/make_oracle_stats.py $W $N $((FIRST + N)) 8 f64 > $D/f64b.log 2>&1 &
else
  SMCDET_ORACLE_OUT=$D/b timeout -k 10 $LIMIT python -u tests/golden/make_oracle_stats.py $W $N $FIRST 8 f32 > $D/f32.log 2>&1 &
fi
p2=$!
# progress for the harness's hang detector
while kill -0 $p1 2>/dev/null || kill -0 $p2 2>/dev/null; do
  sleep 30; date +%T; tail -qn1 $D/*.log
done
wait $p1; wait $p2
echo done
