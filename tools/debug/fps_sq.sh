# SQ counters of one FPS shape (tools/debug/fps_one.py), index-ordered (cull 0) vs culled (cull 1)
export TMPDIR=/tmp
OUT=gpurun_out/fpssq; mkdir -p $OUT
SHAPE=${SHAPE:-"128 16384 512"}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
for c in 0 1; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1)); rm -rf $OUT/c${c}p$i
    timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/c${c}p$i -o run --output-format csv -- python3 tools/debug/fps_one.py $SHAPE $c > $OUT/c${c}p$i.log 2>&1 || { echo "pass c$c p$i failed"; tail -3 $OUT/c${c}p$i.log; exit 1; }
  done
  python3 - $OUT/c${c}p1 $OUT/c${c}p2 <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float); n = collections.Counter()
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "fps" not in r["Kernel_Name"]: continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
c = {k: agg[k] / n[k] for k in agg}
w = c["SQ_WAVES"]; wc = c["SQ_WAVE_CYCLES"]
print("waves %d  wave-cycles/wave %.0f  wait %.2f  winst %.2f  active %.2f  | per wave: valu %.0f salu %.0f lds %.0f smem %.0f branch %.0f | active cycles/wave: valu %.0f lds %.0f sca %.0f misc %.0f  waitinstlds %.0f" % (
    w, wc / w, c["SQ_WAIT_ANY"] / wc, c["SQ_WAIT_INST_ANY"] / wc, c["SQ_ACTIVE_INST_ANY"] / wc,
    c["SQ_INSTS_VALU"] / w, c["SQ_INSTS_SALU"] / w, c["SQ_INSTS_LDS"] / w, c["SQ_INSTS_SMEM"] / w, c["SQ_INSTS_BRANCH"] / w,
    c["SQ_ACTIVE_INST_VALU"] / w, c["SQ_ACTIVE_INST_LDS"] / w, c["SQ_ACTIVE_INST_SCA"] / w, c["SQ_ACTIVE_INST_MISC"] / w, c["SQ_WAIT_INST_LDS"] / w))
PY
done
