#!/bin/bash
# One bench line + rocprofv3 kernel stats per BASELINE config (1 GPU), each step under its own
# time limit; the first failure ends the script.  -> gpurun_out/configs/<cfg>.json, <cfg>_kernel_stats.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/configs
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in ${CONFIGS:-ssg msg pose stress v1}; do
  extra=""
  [ $cfg != ssg ] && extra="--no-cpu-baseline"
  timeout -k 10 400 python bench.py --config $cfg --steps ${STEPS_N:-20} --warmup 5 $extra > $OUT/$cfg.log 2>&1 || { echo "$cfg bench rc=$?"; tail -5 $OUT/$cfg.log; exit 1; }
  grep '^{' $OUT/$cfg.log | tail -1 > $OUT/$cfg.json
  python -c "import json; d=json.load(open('$OUT/$cfg.json')); print('$cfg value', d['value'], 'ms', d['ms_per_step'], 'eager', d.get('eager_value'), 'ref-head', d.get('eager_value_reference_head'), 'fused', (d.get('value_fused') or {}).get('value'), 'frac', (d.get('roofline') or {}).get('frac'))"
  rm -rf $OUT/prof_$cfg
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timer --fused-batches 0 --no-reference-head --no-settled > $OUT/prof_$cfg.log 2>&1 || { echo "$cfg prof rc=$?"; exit 1; }
  cp $(find $OUT/prof_$cfg -name "*kernel_stats.csv" | head -1) $OUT/${cfg}_kernel_stats.csv
  rm -rf $OUT/prof_$cfg
done
