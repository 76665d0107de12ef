#!/bin/bash
# Padded LDS rows of the RV sweep (profiles/r06/ab_pad/pad_rows.patch on the
# c2b1dffc sources, built as the default library): the GPU tests on the padded
# build, a same-box A/B against the unpadded build (smcdet_amd/libsmcdet_hip_head.so
# = `scripts/build_variant.sh head <c2b1dffc mh_kernel.hip>`), and the LDS
# bank-conflict counters of both.  STEPS selects: tests ab pmc.  Result: not
# adopted.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/r06_pad${TAG:-}
mkdir -p $D
STEPS=${STEPS:-"tests ab pmc"}
has() { [[ " $STEPS " == *" $1 "* ]]; }
step() {
  echo "$1 rc=$2"
  if [ "$2" -ne 0 ] && [ "$2" -ne 1 ]; then echo "stopping after $1"; exit "$2"; fi
}
if has tests; then
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest ${TESTS:-tests -m gpu} -v \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
  step tests $?
  grep -E "^FAILED|passed|failed" $D/pytest.log | tail -12
fi
if has ab; then
  LIBS=${LIBS:-head} WORKLOADS=${WORKLOADS:-c2} ROUNDS=${ROUNDS:-3} bash scripts/ab_libs.sh > $D/ab.txt 2>&1
  step ab $?
  cat $D/ab.txt
fi
if has pmc; then
  for tag in cur ${LIBS:-head}; do
    lib=smcdet_amd/libsmcdet_hip.so
    [ "$tag" != cur ] && lib=smcdet_amd/libsmcdet_hip_$tag.so
    SMCDET_ALLOW_STALE=1 SMCDET_HIP_LIB=$PWD/$lib timeout -k 10 240 rocprofv3 \
      --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
      --kernel-include-regex mh_sweep -T -f csv -d $D/pmc_$tag -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-full-run --no-vs-ref --no-c3 \
      --no-legs --no-spread --prewarm-s 0 > $D/pmc_$tag.log 2>&1
    step pmc_$tag $?
  done
  python3 - "$D" ${LIBS:-head} <<'EOF'
import csv, glob, json, sys
from collections import defaultdict
d, tags = sys.argv[1], ["cur"] + sys.argv[2:]
out = {}
for tag in tags:
    f = glob.glob(f"{d}/pmc_{tag}/**/run_counter_collection.csv", recursive=True)[0]
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    names = sorted({c for v in per.values() for c in v})
    out[tag] = {c: sum(v[c] for v in per.values()) / len(per) for c in names}
    out[tag]["dispatches"] = len(per)
print(json.dumps(out, indent=1))
json.dump(out, open(f"{d}/pmc_lds.json", "w"), indent=1)
EOF
fi
