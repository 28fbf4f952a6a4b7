# r04: ball queries on the geometry stream (geometry_bq=1, default) vs in each batch's forward (0)
export TMPDIR=/tmp
OUT=gpurun_out/r04k; mkdir -p $OUT
for i in 1 2; do for v in 1 0; do
  PN2_TUNING=geometry_bq=$v timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/b100_$v$i.log 2>&1 || exit $?
  echo "bq=$v K100 $i $(grep '^{' $OUT/b100_$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  PN2_TUNING=geometry_bq=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b20_$v$i.log 2>&1 || exit $?
  echo "bq=$v K20 $i $(grep '^{' $OUT/b20_$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done; done
for c in msg pose stress; do for v in 1 0; do
  PN2_TUNING=geometry_bq=$v timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c_${c}_$v.log 2>&1 || exit $?
  echo "$c bq=$v K20 $(grep '^{' $OUT/c_${c}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done; done
PN2_TUNING=geometry_bq=0 GPU_MAX_HW_QUEUES=8 FROM_START=1 K=20 timeout -k 10 120 python tools/debug/gpipe_events.py > $OUT/tl_bq0.txt 2>&1 || exit 1
grep -v amdgpu $OUT/tl_bq0.txt | head -24
