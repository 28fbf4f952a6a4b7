#!/bin/bash
# Interleaved A/B of PN2_TUNING settings on the bench (GPU box):
#   VARIANTS="default|dense_lds=0|..." ROUNDS=2 STEPS=20 WARMUP=5 bash tools/tuning_ab.sh
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/tab
mkdir -p $OUT
IFS='|' read -ra VS <<< "${VARIANTS:-default}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "${VS[@]}"; do
    tag=$(echo "$v" | tr -c 'a-zA-Z0-9_' '_')
    if [ "$v" = default ]; then unset PN2_TUNING; else export PN2_TUNING="$v"; fi
    timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} --no-cpu-baseline --no-kernel-timer ${BENCH_ARGS:-} > $OUT/b_${tag}_$r.log 2>&1 || { echo "$v rc=$?"; tail -3 $OUT/b_${tag}_$r.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_${tag}_$r.log') if l.startswith('{')][-1]); print('%-40s round $r: %9.1f clouds/s  %.4f ms/step' % ('$v', d['value'], d['ms_per_step']))"
  done
done
unset PN2_TUNING
