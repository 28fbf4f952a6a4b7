#!/bin/bash
# SQ counter passes (one rocprofv3 run per pass, counters within the per-block limits) over
# the eager bench (each kernel alone on the chip), then a per-kernel summary:
#   CMD="python3 bench.py ..." bash tools/sq_pmc.sh  -> gpurun_out/sqpmc/summary.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sqpmc
rm -rf $OUT && mkdir -p $OUT
export TMPDIR=/tmp
CMD=${CMD:-"python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timer --no-pipeline"}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/sq_summary.py $OUT/p1 $OUT/p2 $OUT/p3 > $OUT/summary.txt && cat $OUT/summary.txt
