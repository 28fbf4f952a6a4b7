#!/bin/bash
# K = 20 with W = 5 (the driver's) vs W = 20 (every pipeline slot replayed before timing),
# interleaved, 3 rounds: does a slot's first replay cost extra?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for w in 5 20; do
    timeout -k 10 300 python bench.py --steps 20 --warmup $w --no-cpu-baseline --no-kernel-timer > gpurun_out/ab/w_$w.log 2>&1 || { echo "$w rc=$?"; exit 1; }
    grep '^{' gpurun_out/ab/w_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('W=$w', d['value'], d['ms_per_step'])"
  done
done
