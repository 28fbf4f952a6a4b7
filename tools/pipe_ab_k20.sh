#!/bin/bash
# A/B of pipeline layouts at the driver's command (K = 20, W = 5; 3 runs) and at K = 100, each
# under its own time limit.  -> gpurun_out/ab/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
run() {  # tag, env assignments..., -- bench args...
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  for k in 20 20 20 100; do
    w=5; [ $k = 100 ] && w=10
    env "${envs[@]}" timeout -k 10 300 python bench.py --steps $k --warmup $w --no-cpu-baseline --no-kernel-timer "$@" > gpurun_out/ab/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -3 gpurun_out/ab/$tag.log; exit 1; }
    grep '^{' gpurun_out/ab/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'K=$k', d['value'], d['ms_per_step'])"
  done
}
run default X=1 --
run heads_compute PN2_TUNING=heads_on_compute=1 --
run no_tail X=1 -- --no-tail
