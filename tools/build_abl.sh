#!/bin/bash
# Timing-only ablation builds of the chain kernel (wrong results; DESIGN.md §4 chains r04):
# pn2/var/abl_<NAME>.so = libpn2.so with sa_chain.hip built with -DPN2_ABL_<flags>.
# Usage: bash tools/build_abl.sh NAME FLAG... (e.g. ALL NOBAR NOEPI NOGATHER NODMA NOLDS)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
P=$ROOT/pointnet-like-pose-estimation_amd
make -s -C $P/csrc -j8
NAME=$1; shift
DEFS=""; for f in "$@"; do DEFS="$DEFS -DPN2_ABL_$f"; done
mkdir -p $P/build/abl $P/pn2/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$ROOT/include -I$P/csrc -Wall -Wno-unused-function $DEFS \
  -c $P/csrc/sa_chain.hip -o $P/build/abl/sa_chain_$NAME.o
OBJS=$(ls $P/build/*.o | grep -v sa_chain.hip.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -Wl,--no-undefined -o $P/pn2/var/abl_$NAME.so $OBJS $P/build/abl/sa_chain_$NAME.o
echo built $P/pn2/var/abl_$NAME.so
