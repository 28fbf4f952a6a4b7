#!/bin/bash
# A/B: bench + kernel stats for the default libpn2.so and each pn2/var/*.so (PN2_TUNING=lib=... override).
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="${BENCH_ARGS:-}"
for lib in default pointnet-like-pose-estimation_amd/pn2/var/*.so; do
  tag=$(basename $lib .so)
  if [ $lib = default ]; then unset PN2_TUNING; else export PN2_TUNING=lib=$PWD/$lib; fi
  for i in 1 2; do
    timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline $ARGS > $OUT/bench_${tag}_$i.log 2>&1 || exit $?
    python - "$tag" $OUT/bench_${tag}_$i.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[2]) if x.startswith('{')][-1]; d=json.loads(l)
print(sys.argv[1], d["value"], d["ms_per_step"], d.get("eager_value"), (d.get("roofline") or {}).get("frac"))
PY
  done
  rm -rf $OUT/prof_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$tag -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timer $ARGS > $OUT/prof_$tag.log 2>&1 || exit $?
  f=$(find $OUT/prof_$tag -name "*kernel_stats.csv" | head -1)
  python - $f <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print("   %-60s %6s %10.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])/1e3))
PY
done
