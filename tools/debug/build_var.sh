#!/bin/bash
# A/B build: libpn2 with one source compiled with extra flags -> tools/var/<name>.so (travels to
# the GPU box; git-ignored)
#   bash tools/debug/build_var.sh <name> <source.hip> <flags...>   (load with PN2_DEBUG_LIB=...)
set -eu
name=$1; src=$2; shift 2
cd "$(dirname "$0")/../../pointnet-like-pose-estimation_amd"
OUT=build/var_$name
mkdir -p $OUT pn2/var ../tools/var
make -s -C csrc >/dev/null
base=$(basename $src)
extra=""
case $base in sa_mlp.hip|sa_chain.hip|sa_dense.hip|linear.hip) ;; *) extra="-ffp-contract=off" ;; esac
[ $base = sa_dense.hip ] && extra="$extra -mllvm -amdgpu-mfma-vgpr-form"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc -Wall -Wno-unused-function \
  $extra "$@" -c csrc/$base -o $OUT/$base.o
objs=$(ls build/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../tools/var/$name.so $objs $OUT/$base.o
echo built tools/var/$name.so
