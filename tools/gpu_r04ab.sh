# r04: FPS block shape 512 x 2 vs the default 256 x 4 (N <= 1024) -- eager and pipelined
# (value = first timed run, value_settled = after ~80 ms of load), interleaved x3
export TMPDIR=/tmp
OUT=gpurun_out/r04ab; mkdir -p $OUT
for i in 1 2 3; do for v in def s512; do for k in 100 20; do
  w=10; [ $k = 20 ] && w=5
  env=""; [ $v = s512 ] && env="PN2_TUNING=fps_threads=512,fps_ppt=2"
  env $env timeout -k 10 300 python3 bench.py --steps $k --warmup $w --no-cpu-baseline --no-kernel-timer > $OUT/b.log 2>&1 || exit $?
  echo "$v K$k $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["value_settled"]["value"], d["eager_value"])')"
done; done; done
