#!/bin/bash
# The driver's bench command (K = 20, W = 5) three times, then one K = 100 run; each under its own
# time limit, the first failure ends the script.  -> gpurun_out/k20/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/k20
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/k20/ssg_$i.log 2>&1 || exit $?
  grep '^{' gpurun_out/k20/ssg_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('k20', d['value'], d['ms_per_step'], d['eager_value'])"
done
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/k20/ssg_k100.log 2>&1 || exit $?
grep '^{' gpurun_out/k20/ssg_k100.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('k100', d['value'], d['ms_per_step'], d['eager_value'])"
