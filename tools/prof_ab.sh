#!/bin/bash
# rocprofv3 kernel stats of the bench under each variant ("tag|env|bench args" per line).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/profab
mkdir -p $OUT
export TMPDIR=/tmp
while IFS='|' read -r tag envs args; do
  [ -z "$tag" ] && continue
  rm -rf $OUT/$tag
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timer $args > $OUT/$tag.log 2>&1 || exit $?
  f=$(find $OUT/$tag -name "*kernel_stats.csv" | head -1)
  echo "== $tag"
  python - $f <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print("   %-70s %6s %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"])/1e3))
PY
done <<< "${VARIANTS}"
