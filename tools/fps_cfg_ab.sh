#!/bin/bash
# A/B of FPS block shapes (PN2_TUNING fps_threads / fps_ppt) inside the pipelined bench and the per-stream timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/fpsab
mkdir -p $OUT
for cfg in ${CFGS:-default 64x16 128x8 256x4}; do
  if [ $cfg = default ]; then unset PN2_TUNING; else export PN2_TUNING=fps_threads=${cfg%x*},fps_ppt=${cfg#*x}; fi
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-kernel-timer ${BENCH_ARGS:-} > $OUT/bench_$cfg.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('$OUT/bench_$cfg.log') if l.startswith('{')][-1]); print('$cfg', d['value'], d['ms_per_step'], d['eager_value'])"
  GEOS=2 timeout -k 10 120 python tools/debug/gpipe_events.py > $OUT/events_$cfg.log 2>&1 || exit $?
  tail -1 $OUT/events_$cfg.log
  awk 'NR>1 && NF>10 {g+=$(NF-2); s+=$(NF-1); h+=$NF; n++} END {printf "   mean geo %.1f sa %.1f head %.1f us\n", g/n, s/n, h/n}' $OUT/events_$cfg.log
done
