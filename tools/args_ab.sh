#!/bin/bash
# Interleaved A/B of bench.py command-line variants (GPU box):
#   VARIANTS="|--slots 10|--geometry-batches 3" ROUNDS=2 STEPS=100 WARMUP=10 bash tools/args_ab.sh
# A variant may start with PN2_TUNING settings: "t:compact_stages=3 --slots 10".
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/aab
mkdir -p $OUT
IFS='|' read -ra VS <<< "${VARIANTS:-}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "${VS[@]}"; do
    tag=$(echo "x$v" | tr -c 'a-zA-Z0-9_' '_')
    tun=""; args="$v"
    case "$v" in t:*) tun="${v%% *}"; tun="${tun#t:}"; args="${v#* }"; [ "$args" = "$v" ] && args="";; esac
    if [ -n "$tun" ]; then export PN2_TUNING="$tun"; else unset PN2_TUNING; fi
    timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup ${WARMUP:-10} --no-cpu-baseline --no-kernel-timer ${BENCH_ARGS:-} $args > $OUT/b_${tag}_$r.log 2>&1 || { echo "$v rc=$?"; tail -3 $OUT/b_${tag}_$r.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_${tag}_$r.log') if l.startswith('{')][-1]); print('%-44s round $r: %9.1f clouds/s  %.4f ms/step' % ('[$v]', d['value'], d['ms_per_step']))"
  done
done
unset PN2_TUNING
