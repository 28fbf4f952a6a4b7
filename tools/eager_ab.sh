#!/bin/bash
# Eager forward A/B (bench --no-pipeline): default vs PN2_TUNING=geometry_stream=1, interleaved, 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for v in 0 1; do
    PN2_TUNING=geometry_stream=$v timeout -k 10 300 python bench.py --no-pipeline --steps 100 --warmup 10 --no-cpu-baseline --no-kernel-timer > gpurun_out/ab/e_$v.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    grep '^{' gpurun_out/ab/e_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('geometry_stream=$v', d['value'], d['ms_per_step'])"
  done
done
