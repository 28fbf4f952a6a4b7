#!/bin/bash
# A/B of pipeline options (each line of $VARIANTS: "tag|env|bench args") on the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pipeab
mkdir -p $OUT
while IFS='|' read -r tag envs args; do
  [ -z "$tag" ] && continue
  for i in 1 2; do
    env $envs timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-kernel-timer $args > $OUT/bench_${tag}_$i.log 2>&1 || exit $?
    python -c "import json; d=json.loads([l for l in open('$OUT/bench_${tag}_$i.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'], d['eager_value'])"
  done
done <<< "${VARIANTS:-base|X=1|
slots4|X=1|--slots 4
splitlast|PN2_TUNING=pipe_split_last=1|
splitlast4|PN2_TUNING=pipe_split_last=1|--slots 4}"
