#!/bin/bash
# Tile pass (temper -> reweight -> systematic indices): phase cycles from the
# trace build at 512 and 256 threads, then a same-box A/B of the C2 bench
# line with the 512-thread (default) and 256-thread tile kernel
# (SMCDET_TILE_THREADS), alternating, and the rocprofv3 kernel trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/tile_nt
mkdir -p $D
for nt in 512 256; do
  SMCDET_TILE_THREADS=$nt SMCDET_ALLOW_STALE=1 timeout -k 10 200 python scripts/trace_phases.py 5 \
    > $D/phases_$nt.json 2> $D/phases_$nt.err
  rc=$?; echo "phases $nt rc=$rc"; [ $rc -ne 0 ] && { tail -5 $D/phases_$nt.err; exit $rc; }
  python - $D/phases_$nt.json << 'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k in ("step2", "step3", "step4"):
    print(k, {a: round(b) for a, b in d[k]["tile_cycles"].items()})
PY
done
Q="--no-cpu-baseline --no-full-run --no-vs-ref --no-spread --no-c3"
for rep in 1 2 3; do
  for nt in 512 256; do
    SMCDET_TILE_THREADS=$nt timeout -k 10 200 python bench.py $Q > $D/c2_nt${nt}_r$rep.json 2> $D/c2_nt${nt}_r$rep.err
    rc=$?; [ $rc -ne 0 ] && { echo "bench $nt rc=$rc"; exit $rc; }
    python - $D/c2_nt${nt}_r$rep.json $nt $rep << 'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("nt", sys.argv[2], "rep", sys.argv[3], "value %.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"],
      "mh_ms %.4f" % d["roofline"]["kernel_ms"], flush=True)
PY
  done
done
for nt in 512 256; do
  SMCDET_TILE_THREADS=$nt timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $D/trace_$nt -o run -- \
    python3 bench.py $Q --steps 20 > $D/trace_$nt.log 2>&1
  rc=$?; echo "trace $nt rc=$rc"; [ $rc -ne 0 ] && exit $rc
  tr=$(find $D/trace_$nt -name 'run_kernel_trace.csv' | head -1)
  python scripts/step_attribution.py "$tr" --json $D/step_attribution_$nt.json | grep -E "tile_us|sweep_us"
done
