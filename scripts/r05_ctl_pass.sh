set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/ctl
mkdir -p $D
timeout -k 10 120 python scripts/lib_outputs.py $D/cur.npz > $D/out_cur.log 2>&1 || { tail -5 $D/out_cur.log; exit 1; }
SMCDET_ALLOW_STALE=1 SMCDET_HIP_LIB=$PWD/smcdet_amd/libsmcdet_hip_${V:-ctl}.so timeout -k 10 120 python scripts/lib_outputs.py $D/v.npz > $D/out_v.log 2>&1 || { tail -5 $D/out_v.log; exit 1; }
python scripts/lib_outputs.py --compare $D/cur.npz $D/v.npz
LIBS="${V:-ctl}" SLOTS=5 REPS=3 bash scripts/ab_mb_libs.sh || exit 1
LIBS="${V:-ctl}" WORKLOADS="${WL:-c4}" ROUNDS=2 BENCH_ARGS="--steps 10 --warmup 2" bash scripts/ab_libs.sh
