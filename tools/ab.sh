#!/bin/bash
# The one interleaved A/B runner (GPU box).  A variant is a set of bench.py arguments, optionally
# led by PN2_TUNING settings ("t:fps_red=2,fps_mid=256 --slots 16"); the empty variant is the
# default build and launch.  Variants are separated by '|' and run interleaved, ROUNDS times.
#
#   VARIANTS="|t:fps_red=2" ROUNDS=3 STEPS=20 WARMUP=5 MODE=bench bash tools/ab.sh
#
# MODE=bench  one bench line per (variant, round): value (and eager_value) -> gpurun_out/ab/
# MODE=eager  the same with --no-pipeline (the eager forward is the timed loop)
# MODE=prof   rocprofv3 --kernel-trace --stats of an eager bench per variant -> kstats per variant
# MODE=pmc    FETCH_SIZE and WRITE_SIZE passes (one counter per run) of the eager bench per
#             variant -> HBM bytes per MLP call (tools/pmc_traffic.py)
# CFG (default ssg) is the bench config; BENCH_ARGS go to every run.  Every GPU step has its own
# time limit; the first failure ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp
MODE=${MODE:-bench}
CFG=${CFG:-ssg}
IFS='|' read -ra VS <<< "${VARIANTS:-}"
[ ${#VS[@]} -eq 0 ] && VS=("")
split() {  # variant -> $tun (PN2_TUNING) and $args (bench arguments)
  local v="$1"; tun=""; args="$v"
  case "$v" in t:*) tun="${v%% *}"; tun="${tun#t:}"; args="${v#* }"; [ "$args" = "$v" ] && args="";; esac
}
rounds=${ROUNDS:-2}
[ "$MODE" = prof ] || [ "$MODE" = pmc ] && rounds=1
for r in $(seq 1 $rounds); do
  for v in "${VS[@]}"; do
    tag=$(echo "x$v" | tr -c 'a-zA-Z0-9_' '_')
    split "$v"
    if [ -n "$tun" ]; then export PN2_TUNING="$tun"; else unset PN2_TUNING; fi
    base="--config $CFG --no-cpu-baseline --no-kernel-timer ${BENCH_ARGS:-}"
    case "$MODE" in
      bench|eager)
        extra=""; [ "$MODE" = eager ] && extra="--no-pipeline --no-reference-head"
        timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} $base $extra $args > $OUT/b_${tag}_$r.log 2>&1 \
          || { echo "[$v] rc=$?"; tail -5 $OUT/b_${tag}_$r.log; exit 1; }
        python -c "import json; d=json.loads([l for l in open('$OUT/b_${tag}_$r.log') if l.startswith('{')][-1]); print('%-48s round $r: value %9.1f  eager %9.1f  ref-head %s' % ('[$v]', d['value'], d['eager_value'], d.get('eager_value_reference_head')))"
        ;;
      prof)
        rm -rf $OUT/prof_$tag
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$tag -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-pipeline --no-reference-head --fused-batches 0 $base $args > $OUT/prof_$tag.log 2>&1 \
          || { echo "[$v] prof rc=$?"; tail -5 $OUT/prof_$tag.log; exit 1; }
        python tools/kstats.py $OUT/prof_$tag > $OUT/kstats_$tag.txt
        rm -rf $OUT/prof_$tag
        echo "== [$v]"; head -16 $OUT/kstats_$tag.txt
        ;;
      pmc)
        for c in FETCH_SIZE WRITE_SIZE; do
          rm -rf $OUT/pmc_${tag}_$c
          timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/pmc_${tag}_$c -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-pipeline --no-reference-head --fused-batches 0 $base $args > $OUT/pmc_${tag}_$c.log 2>&1 \
            || { echo "[$v] pmc $c rc=$?"; tail -5 $OUT/pmc_${tag}_$c.log; exit 1; }
        done
        python3 tools/pmc_traffic.py $OUT/pmc_${tag}_FETCH_SIZE $OUT/pmc_${tag}_WRITE_SIZE --config $CFG --forwards 7 --no-save > $OUT/pmc_summary_$tag.txt 2>&1
        echo "== [$v]"; grep -E "sa_chain|compact_scan|dense_|fps|ball_query|per_call" $OUT/pmc_summary_$tag.txt
        ;;
      *) echo "unknown MODE=$MODE"; exit 2;;
    esac
  done
done
unset PN2_TUNING
