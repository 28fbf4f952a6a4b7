# r04: bench warm-up order (pipelined warm-up before the eager one) A/B
export TMPDIR=/tmp
OUT=gpurun_out/r04u; mkdir -p $OUT
for i in 1 2 3; do for v in 0 1; do
  for k in 100 20; do
    w=10; [ $k = 20 ] && w=5
    PN2_BENCH_PIPE_FIRST=$v timeout -k 10 300 python3 bench.py --steps $k --warmup $w --no-cpu-baseline > $OUT/b.log 2>&1 || exit $?
    echo "pipe_first=$v K$k $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"])')"
  done
done; done
