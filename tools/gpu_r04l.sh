# r04: the three co-bottleneck streams -- ball queries off the geometry stream combined with the
# head placement (second tail stream / heads on the compute streams)
export TMPDIR=/tmp
OUT=gpurun_out/r04l; mkdir -p $OUT
VS="default geometry_bq=0,tail_streams=2 geometry_bq=0,heads_on_compute=1 tail_streams=2 heads_on_compute=1"
for i in 1 2; do for v in $VS; do
  t=$v; [ $v = default ] && t=""
  for k in 100 20; do
    w=10; [ $k = 20 ] && w=5
    PN2_TUNING=$t timeout -k 10 300 python3 bench.py --steps $k --warmup $w --no-cpu-baseline > $OUT/b_${k}_$i.log 2>&1 || exit $?
    echo "$v K$k $i $(grep '^{' $OUT/b_${k}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done; done
