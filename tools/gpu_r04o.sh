# r04: CU-partitioned geometry stream (FPS away from the chains' SIMDs) vs shared CUs
export TMPDIR=/tmp
OUT=gpurun_out/r04o; mkdir -p $OUT
for i in 1 2; do for g in 0 32 64; do
  for k in 100 20; do
    w=10; [ $k = 20 ] && w=5
    timeout -k 10 300 python3 bench.py --steps $k --warmup $w --no-cpu-baseline --geometry-cus $g > $OUT/b.log 2>&1 || exit $?
    echo "gcus=$g K$k $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done; done
