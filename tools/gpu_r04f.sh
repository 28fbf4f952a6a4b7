# r04: FPS -- coalesced packed-record write (traffic), culled shapes with fewer waves per SIMD
export TMPDIR=/tmp
OUT=gpurun_out/r04f; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fps_cull.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_fps.py --cull=0,1,102444,51284,51362,51248,25684 --tag cull3 > $OUT/fps.log 2>&1 || exit $?
grep -v amdgpu $OUT/fps.log | cut -c1-110
for c in 0 102444 51284 51362; do
  rm -rf $OUT/pmc_$c
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE -d $OUT/pmc_$c -o run --output-format csv -- python3 tools/debug/fps_one.py 128 16384 512 $c > $OUT/pmc_$c.log 2>&1 || exit $?
  python3 - $OUT/pmc_$c $c <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fps" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: "%.1f" % (sum(v) / len(v)) for k, v in agg.items()}, "(KB per dispatch, per guide units)")
PY
done
