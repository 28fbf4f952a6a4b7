# r04: dense tile width in the pipeline: dense_minwg 256 (default) vs 128 (sa3's first layer in
# 64-column tiles, 128 workgroups)
export TMPDIR=/tmp
OUT=gpurun_out/r04q; mkdir -p $OUT
for i in 1 2 3; do for v in default dense_minwg=128; do
  t=$v; [ $v = default ] && t=""
  for k in 100 20; do
    w=10; [ $k = 20 ] && w=5
    PN2_TUNING=$t timeout -k 10 300 python3 bench.py --steps $k --warmup $w --no-cpu-baseline > $OUT/b.log 2>&1 || exit $?
    echo "$v K$k $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"])')"
  done
done; done
