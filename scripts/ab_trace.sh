set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/abt; mkdir -p $D
Q="--no-cpu-baseline --no-full-run --no-vs-ref --no-spread --no-c3 --steps 20"
for r in 1 2; do
for tag in cur old; do
  lib=smcdet_amd/libsmcdet_hip.so; [ $tag = old ] && lib=smcdet_amd/libsmcdet_hip_old.so
  SMCDET_ALLOW_STALE=1 SMCDET_HIP_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $D/${tag}_$r -o run -- python3 bench.py $Q > $D/${tag}_$r.log 2>&1 || { echo "$tag rc=$?"; exit 1; }
  tr=$(find $D/${tag}_$r -name 'run_kernel_trace.csv' | head -1)
  echo "$tag r$r $(python scripts/step_attribution.py $tr --json $D/sa_${tag}_$r.json | grep -E 'tile_us|sweep_us' | tr '\n' ' ' | cut -c1-220)"
done
done
