#!/bin/bash
# Tail stream priority A/B at the driver's command (K = 20, W = 5) and K = 100, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for v in 0 1; do
    for k in 20 100; do
      w=5; [ $k = 100 ] && w=10
      PN2_TUNING=tail_prio=$v timeout -k 10 300 python bench.py --steps $k --warmup $w --no-cpu-baseline --no-kernel-timer > gpurun_out/ab/t_$v.log 2>&1 || { echo "$v rc=$?"; exit 1; }
      grep '^{' gpurun_out/ab/t_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tail_prio=$v K=$k', d['value'], d['ms_per_step'])"
    done
  done
done
