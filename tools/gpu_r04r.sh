# r04: eager forward with layer i+1's FPS + ball query on a side stream (geometry_stream=1)
export TMPDIR=/tmp
OUT=gpurun_out/r04r; mkdir -p $OUT
for i in 1 2; do for v in default geometry_stream=1; do
  t=$v; [ $v = default ] && t=""
  for c in ssg msg pose stress; do
    PN2_TUNING=$t timeout -k 10 300 python3 bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timer > $OUT/b.log 2>&1 || exit $?
    echo "$v $c $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"])')"
  done
done; done
