#!/bin/bash
# MFMA utilisation from counters, per BASELINE config: one SQ pass per
# config over the eager bench (each kernel alone on the chip) -> gpurun_out/sqmfma/sq_summary_<cfg>.txt
# and sq_mfma_<cfg>.json; bench.py reads profiles/sq_mfma.json (merged by tools/sq_mfma_merge.py).
#   CONFIGS="ssg msg pose stress v1" bash tools/sq_mfma.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sqmfma
mkdir -p $OUT
export TMPDIR=/tmp
P="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for cfg in ${CONFIGS:-ssg}; do
  rm -rf $OUT/p_$cfg
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timer --no-pipeline > $OUT/p_$cfg.log 2>&1 || { echo "sq pass $cfg rc=$?"; tail -5 $OUT/p_$cfg.log; exit 1; }
  python3 tools/sq_summary.py $OUT/p_$cfg --json $OUT/sq_mfma_$cfg.json > $OUT/sq_summary_$cfg.txt
  head -8 $OUT/sq_summary_$cfg.txt
done
