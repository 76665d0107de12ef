#!/bin/bash
# Builds smcdet_amd/libsmcdet_hip_<tag>.so with one kernel source replaced by a
# variant file (same-box A/B with scripts/ab_libs.sh):
#   scripts/build_variant.sh <tag> <variant.hip> [replaced source, default mh_kernel.hip]
set -eu
cd "$(dirname "$0")/.."
tag=$1; src=$2; rep=${3:-mh_kernel.hip}
C=smcdet_amd/csrc
make -s $C/common.o $C/model_kernels.o $C/mh_kernel.o $C/mala_kernel.o $C/chain_kernel.o $C/smc_kernels.o $C/agg_kernel.o
cp "$src" $C/_variant_$tag.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result \
  -c $C/_variant_$tag.hip -o $C/_variant_$tag.o
objs=""
for o in common model_kernels mh_kernel mala_kernel chain_kernel smc_kernels agg_kernel; do
  if [ "$o.hip" = "$rep" ]; then objs="$objs $C/_variant_$tag.o"; else objs="$objs $C/$o.o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o smcdet_amd/libsmcdet_hip_$tag.so $objs
rm -f $C/_variant_$tag.hip $C/_variant_$tag.o
echo built smcdet_amd/libsmcdet_hip_$tag.so
