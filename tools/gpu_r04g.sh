# r04: FPS traffic (FETCH_SIZE / WRITE_SIZE passes) of the STRESS launch, index-ordered and culled
export TMPDIR=/tmp
OUT=gpurun_out/r04g; mkdir -p $OUT
for c in 0 102444; do for P in FETCH_SIZE WRITE_SIZE; do
  rm -rf $OUT/pmc_${c}_$P
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/pmc_${c}_$P -o run --output-format csv -- python3 tools/debug/fps_one.py 128 16384 512 $c > $OUT/pmc_${c}_$P.log 2>&1 || exit $?
  python3 - $OUT/pmc_${c}_$P $c <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fps" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: "%.1f" % (sum(v) / len(v)) for k, v in agg.items()}, "(per dispatch, raw counter units)")
PY
done; done
