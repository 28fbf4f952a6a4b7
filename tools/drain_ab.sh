#!/bin/bash
# Drain A/B at the driver's command (K = 20, W = 5) and K = 100: the last PN2_DRAIN_HEADS
# batches' heads on their compute streams (0 = all on the tail stream), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for v in ${DRAINS:-0 2 4}; do
    for k in ${KS:-20}; do
      PN2_TUNING=drain_heads=$v timeout -k 10 300 python bench.py --steps $k --warmup 5 --no-cpu-baseline --no-kernel-timer > gpurun_out/ab/d_$v.log 2>&1 || { echo "$v rc=$?"; exit 1; }
      grep '^{' gpurun_out/ab/d_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('drain=$v K=$k', d['value'], d['ms_per_step'])"
    done
  done
done
