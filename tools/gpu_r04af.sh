# r04: dense_lds_mincin -- SSG eager (in-process A/B) and PointNet-v1's eager forward
export TMPDIR=/tmp
OUT=gpurun_out/r04af; mkdir -p $OUT
EAGER_AB_SET=profile timeout -k 10 300 python tools/debug/eager_ab.py 3 2>&1 | grep "clouds/s\|differs" || exit 1
for i in 1 2; do for m in 256 128 0; do
  PN2_TUNING=dense_lds_mincin=$m timeout -k 10 300 python3 bench.py --config v1 --steps 50 --no-cpu-baseline --no-kernel-timer > $OUT/b.log 2>&1 || exit $?
  echo "v1 mincin=$m $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"])')"
done; done
