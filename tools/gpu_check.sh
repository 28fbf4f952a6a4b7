#!/bin/bash
# GPU-box runner: tests, smoke, bench, rocprofv3 kernel stats.  Every GPU step has its own
# time limit; any exit that is not 0 (or 1 = ordinary pytest test failure) ends the script
# before another GPU step starts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEPS="${STEPS:-pytest smoke bench prof}"
ok() { local rc=$1 what=$2; echo "[gpu_check] $what rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_check] stopping after $what (rc=$rc)"; exit $rc; fi; }
for s in $STEPS; do
  case $s in
    pytest)
      timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout=600 ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; ok $? pytest
      tail -30 $OUT/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; ok $? smoke
      tail -5 $OUT/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-100} --warmup 10 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; ok $? bench
      tail -3 $OUT/bench.log ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timer ${BENCH_ARGS:-} > $OUT/prof.log 2>&1; ok $? prof
      find $OUT/prof -name "*kernel_stats.csv" | head -3 ;;
    pmc)
      # one counter per pass (FETCH_SIZE and WRITE_SIZE do not fit one gfx950 TCC pass);
      # eager launch so every kernel runs on the full chip, as the kernel timer measures it
      for cfg in ${PMC_CONFIGS:-ssg}; do
        for c in FETCH_SIZE WRITE_SIZE; do
          rm -rf $OUT/pmc_${cfg}_$c
          timeout -k 10 300 rocprofv3 --pmc $c -d $OUT/pmc_${cfg}_$c -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timer --no-pipeline > $OUT/pmc_${cfg}_$c.log 2>&1; ok $? pmc_${cfg}_$c
        done
        python tools/pmc_traffic.py $OUT/pmc_${cfg}_FETCH_SIZE $OUT/pmc_${cfg}_WRITE_SIZE --config $cfg --forwards 7 > $OUT/pmc_summary_$cfg.txt 2>&1
        head -3 $OUT/pmc_summary_$cfg.txt
      done
      cp profiles/pmc_traffic.json $OUT/pmc_traffic.json ;;
    *) echo "unknown step $s" ;;
  esac
done
