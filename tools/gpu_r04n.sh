# r04: FPS footprint in the pipeline (SSG): 4 waves x 4 points (default) vs 2 x 8 vs 1 x 16
export TMPDIR=/tmp
OUT=gpurun_out/r04n; mkdir -p $OUT
VS="default fps_threads=128,fps_ppt=8 fps_threads=64,fps_ppt=16"
for i in 1 2; do for v in $VS; do
  t=$v; [ $v = default ] && t=""
  for k in 100 20; do
    w=10; [ $k = 20 ] && w=5
    PN2_TUNING=$t timeout -k 10 300 python3 bench.py --steps $k --warmup $w --no-cpu-baseline > $OUT/b.log 2>&1 || exit $?
    echo "$v K$k $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"])')"
  done
done; done
