# r04: two geometry streams (consecutive groups' geometry in parallel; 8 hardware queues now)
export TMPDIR=/tmp
OUT=gpurun_out/r04s; mkdir -p $OUT
for i in 1 2 3; do for gs in 1 2; do
  for k in 100 20; do
    w=10; [ $k = 20 ] && w=5
    timeout -k 10 300 python3 bench.py --steps $k --warmup $w --no-cpu-baseline --geometry-streams $gs > $OUT/b.log 2>&1 || exit $?
    echo "gs=$gs K$k $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done; done
