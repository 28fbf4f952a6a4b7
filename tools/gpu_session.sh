#!/bin/bash
# GPU-box runner for one A/B iteration:
#   PYTEST=all (optional: the whole -m gpu suite first) or PYTEST_K="expr" (a -k selection)
#   KT="tag:tuning|tag:tuning" (optional: eager rocprofv3 kernel traces per PN2_TUNING variant,
#                                summarised by tools/kstats.py)
#   VARIANTS=... (optional: interleaved bench A/B, tools/ab.sh syntax), STEPS, WARMUP, ROUNDS
#   BENCH_ARGS=... (passed to every bench run)
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sess
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "${PYTEST:-}" ] || [ -n "${PYTEST_K:-}" ]; then
  if [ -n "${PYTEST_K:-}" ]; then sel=(-k "$PYTEST_K"); else sel=(); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${sel[@]}" > $OUT/pytest.log 2>&1
  rc=$?; tail -4 $OUT/pytest.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
if [ -n "${KT:-}" ]; then
  IFS='|' read -ra KS <<< "$KT"
  for kv in "${KS[@]}"; do
    tag=${kv%%:*}; tun=${kv#*:}
    rm -rf $OUT/kt_$tag
    if [ -n "$tun" ]; then export PN2_TUNING="$tun"; else unset PN2_TUNING; fi
    timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt_$tag -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timer --no-pipeline ${BENCH_ARGS:-} > $OUT/kt_$tag.log 2>&1
    rc=$?; unset PN2_TUNING; [ $rc -ne 0 ] && { echo "kt $tag rc=$rc"; tail -5 $OUT/kt_$tag.log; exit $rc; }
    python tools/kstats.py $OUT/kt_$tag > $OUT/kstats_$tag.txt
    echo "== eager $tag"; head -14 $OUT/kstats_$tag.txt
  done
fi
if [ -n "${VARIANTS:-}" ]; then
  bash tools/ab.sh || exit $?
fi
