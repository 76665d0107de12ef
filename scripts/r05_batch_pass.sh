set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/batch
mkdir -p $D
timeout -k 10 120 python scripts/lib_outputs.py $D/cur.npz > $D/out_cur.log 2>&1 || { tail -5 $D/out_cur.log; exit 1; }
SMCDET_ALLOW_STALE=1 SMCDET_HIP_LIB=$PWD/smcdet_amd/libsmcdet_hip_bG.so timeout -k 10 120 python scripts/lib_outputs.py $D/bG.npz > $D/out_bG.log 2>&1 || { tail -5 $D/out_bG.log; exit 1; }
python scripts/lib_outputs.py --compare $D/cur.npz $D/bG.npz
LIBS="bG bH" SLOTS=5 REPS=3 bash scripts/ab_mb_libs.sh || exit 1
LIBS="bF bG bH" WORKLOADS=c4 ROUNDS=2 BENCH_ARGS="--steps 10 --warmup 2" bash scripts/ab_libs.sh
