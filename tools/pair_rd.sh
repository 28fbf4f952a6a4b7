#!/bin/bash
# dense_pair_kernel weight-stream depth A/B (tools/debug/eager_run.py under rocprofv3 per build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pair_rd
mkdir -p $OUT
export TMPDIR=/tmp
for rd in ${RDS:-4 8 12 16}; do
  bash tools/debug/build_var.sh rd$rd csrc/sa_dense.hip -DPN2_PAIR_RD=$rd > /dev/null 2>&1 || { echo build rd$rd failed; exit 1; }
  rm -rf $OUT/rd$rd
  PN2_DEBUG_LIB=pointnet-like-pose-estimation_amd/pn2/var/rd$rd.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/rd$rd -o run --output-format csv -- python3 tools/debug/eager_run.py > $OUT/rd$rd.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rd$rd rc=$rc"; tail -5 $OUT/rd$rd.log; exit $rc; }
  echo "rd$rd: $(grep eager $OUT/rd$rd.log)"
  python tools/kstats.py $OUT/rd$rd | grep -E "pair|dense_lds" ; rm -rf $OUT/rd$rd
done
