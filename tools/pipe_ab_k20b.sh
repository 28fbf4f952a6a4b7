#!/bin/bash
# Interleaved A/B at the driver's command (K = 20, W = 5): default layout vs --no-tail, 5 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for r in 1 2 3 4 5; do
  for v in default no_tail; do
    a=""; [ $v = no_tail ] && a="--no-tail"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timer $a > gpurun_out/ab/b_$v.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    grep '^{' gpurun_out/ab/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['eager_value'])"
  done
done
