#!/bin/bash
# HBM traffic per kernel for tuning variants (FETCH_SIZE and WRITE_SIZE passes of the eager
# bench per variant, PN2_TUNING set; nothing saved under profiles/):
#   VARIANTS="base:|nopool:compact_pool=8" CFG=ssg bash tools/pmc_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmcab
mkdir -p $OUT
export TMPDIR=/tmp
CFG=${CFG:-ssg}
IFS='|' read -ra VS <<< "${VARIANTS:-base:}"
for kv in "${VS[@]}"; do
  tag=${kv%%:*}; tun=${kv#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf $OUT/${tag}_$c
    if [ -n "$tun" ]; then export PN2_TUNING="$tun"; else unset PN2_TUNING; fi
    timeout -k 10 300 rocprofv3 --pmc $c -d $OUT/${tag}_$c -o run --output-format csv -- python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timer --no-pipeline > $OUT/${tag}_$c.log 2>&1
    rc=$?; unset PN2_TUNING; [ $rc -ne 0 ] && { echo "pmc $tag $c rc=$rc"; tail -5 $OUT/${tag}_$c.log; exit $rc; }
  done
  python3 tools/pmc_traffic.py $OUT/${tag}_FETCH_SIZE $OUT/${tag}_WRITE_SIZE --config $CFG --forwards 7 --no-save > $OUT/summary_$tag.txt 2>&1
  echo "== $tag ($tun)"; grep -E "sa_chain|compact_scan|u_table|dense_lds|dense_split|per_call" $OUT/summary_$tag.txt
done
