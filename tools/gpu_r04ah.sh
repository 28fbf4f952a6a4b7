# r04 final: the driver's command five times on one box (value, value_settled, eager_value)
export TMPDIR=/tmp
OUT=gpurun_out/r04ah; mkdir -p $OUT
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b$i.log 2>&1 || exit $?
  echo "K20 $i $(grep '^{' $OUT/b$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["value_settled"]["value"], d["eager_value"])')"
done
