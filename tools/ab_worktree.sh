#!/bin/bash
# A/B of git worktrees under _ab/ (built in place) against the working tree on one GPU box,
# interleaved: VARIANTS="e98 e2b1ddd ." REPS=2 -> gpurun_out/ab/<variant>_<rep>.log
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab
F=${BENCH_FLAGS:-"--steps 20 --warmup 5 --no-cpu-baseline --fused-batches 0 --no-reference-head --no-kernel-timer"}
for i in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS}; do
    d=_ab/$v; [ "$v" = "." ] && d=.
    tag=$(echo $v | tr -d './')_$i; [ "$v" = "." ] && tag=head_$i
    (cd $d && timeout -k 10 300 python bench.py $F > $GRAFT_REPO_ROOT/gpurun_out/ab/$tag.log 2>&1) || exit 1
    grep '^{' gpurun_out/ab/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['eager_value'])"
  done
done
