#!/bin/bash
# Same-box A/B of the round-3 tree (exported to _r03/ with `git archive
# 4988c04`, built there; not part of the repository) against HEAD: the C2
# bench line, C4 and the C3 64-tile line, alternating, ROUNDS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r03r04; mkdir -p $D
Q0="--no-cpu-baseline --no-full-run --no-vs-ref --no-spread"
for r in $(seq 1 ${ROUNDS:-3}); do
  for tree in r04 r03; do
    dir=.; Q="$Q0 --no-c3"
    [ $tree = r03 ] && { dir=_r03; Q="$Q0"; }  # (round 3's bench had no --no-c3)
    for wl in "c2" "c4" "c2 --total-tiles 64"; do
      tag=$(echo "$wl" | tr ' ' '_' | tr -d '-')
      (cd $dir && timeout -k 10 300 python bench.py --workload $wl $Q) > $D/${tree}_${tag}_r$r.log 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "$tree $wl rc=$rc"; tail -5 $D/${tree}_${tag}_r$r.log; exit $rc; }
      python - $D/${tree}_${tag}_r$r.log "$tree" "$wl" $r << 'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], sys.argv[3], "r" + sys.argv[4], "%.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"],
      "mh_ms", round(d.get("roofline", {}).get("kernel_ms") or 0, 4), flush=True)
PY
    done
  done
done
