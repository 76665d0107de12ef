set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/gap
for tag in cur ntrate; do
  lib=$PWD/smcdet_amd/libsmcdet_hip.so; [ $tag != cur ] && lib=$PWD/smcdet_amd/libsmcdet_hip_$tag.so
  SMCDET_ALLOW_STALE=1 SMCDET_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d gpurun_out/gap/$tag -o run -- python3 scripts/gap_probe.py 10 > gpurun_out/gap/$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/gap/$tag.log; exit 1; }
  f=$(find gpurun_out/gap/$tag -name "*kernel_trace.csv" | head -1)
  echo "== $tag"; python scripts/gap_summary.py $f 33
done
