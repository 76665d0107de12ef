set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/pk
mkdir -p $D
timeout -k 10 120 python scripts/lib_outputs.py $D/new.npz > $D/out_new.log 2>&1 || { tail -5 $D/out_new.log; exit 1; }
SMCDET_ALLOW_STALE=1 SMCDET_HIP_LIB=$PWD/smcdet_amd/libsmcdet_hip_head.so timeout -k 10 120 python scripts/lib_outputs.py $D/head.npz > $D/out_head.log 2>&1 || { tail -5 $D/out_head.log; exit 1; }
python scripts/lib_outputs.py --compare $D/head.npz $D/new.npz
LIBS=head SLOTS=5 REPS=3 bash scripts/ab_mb_libs.sh || exit 1
LIBS=head WORKLOADS=c4 ROUNDS=2 BENCH_ARGS="--steps 10 --warmup 2" bash scripts/ab_libs.sh
