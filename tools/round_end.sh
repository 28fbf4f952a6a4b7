#!/bin/bash
# Round-end record on one GPU box: GPU tests, smoke, the default bench (K = 100), the driver's
# command three times (K = 20, W = 5), and rocprofv3 kernel stats of the pipelined and of the
# eager launch -> gpurun_out/end/.  Every GPU step has its own time limit; the first failure
# ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/end
mkdir -p $OUT
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[round_end] $what rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
step $? pytest; tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
step $? smoke; tail -2 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_default.log 2>&1
step $? bench_default; grep '^{' $OUT/bench_default.log | tail -1 > $OUT/bench_default.json
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_k20_$i.log 2>&1
  step $? bench_k20_$i; grep '^{' $OUT/bench_k20_$i.log | tail -1 > $OUT/bench_k20_$i.json
done
python - <<'PY'
import json
for f in ["bench_default"] + ["bench_k20_%d" % i for i in (1, 2, 3)]:
    d = json.load(open("gpurun_out/end/%s.json" % f))
    print(f, d["value"], d["ms_per_step"], (d.get("value_settled") or {}).get("value"),
          d.get("eager_value"), d["roofline"]["frac"], (d.get("cpu_baseline") or {}).get("value"))
PY
rm -rf $OUT/prof_pipe $OUT/prof_eager
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_pipe -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timer > $OUT/prof_pipe.log 2>&1
step $? prof_pipe
cp $(find $OUT/prof_pipe -name "*kernel_stats.csv" | head -1) $OUT/pipelined_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_eager -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timer --no-pipeline > $OUT/prof_eager.log 2>&1
step $? prof_eager
cp $(find $OUT/prof_eager -name "*kernel_stats.csv" | head -1) $OUT/eager_kernel_stats.csv
python tools/kstats.py $OUT/prof_eager > $OUT/kstats_eager.txt
head -16 $OUT/kstats_eager.txt
rm -rf $OUT/prof_pipe $OUT/prof_eager
