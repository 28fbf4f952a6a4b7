#!/bin/bash
# Diagnostic build: libpn2 with timeline stamps in the dense layer kernel (-DPN2_DENSE_STAMPS)
# -> pointnet-like-pose-estimation_amd/pn2/var/dstamps.so (load with PN2_DEBUG_LIB=...)
set -eu
bash "$(dirname "$0")/build_var.sh" dstamps csrc/sa_dense.hip -DPN2_DENSE_STAMPS
