#!/bin/bash
# Diagnostic build: libpn2 with timeline stamps in the SA chain kernel (-DPN2_CHAIN_STAMPS)
# -> pointnet-like-pose-estimation_amd/pn2/var/stamps.so (load with PN2_DEBUG_LIB=...)
set -eu
cd "$(dirname "$0")/../../pointnet-like-pose-estimation_amd"
OUT=build/stamps
mkdir -p $OUT pn2/var
make -s -C csrc >/dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc -Wall -Wno-unused-function \
  -DPN2_CHAIN_STAMPS -c csrc/sa_chain.hip -o $OUT/sa_chain.hip.o
objs=$(ls build/*.o | grep -v sa_chain.hip.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o pn2/var/stamps.so $objs $OUT/sa_chain.hip.o
echo built pn2/var/stamps.so
