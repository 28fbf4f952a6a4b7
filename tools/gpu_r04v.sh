# r04: why tools/debug/host_bound.py reads ~149k at K = 100 and bench.py ~139k
export TMPDIR=/tmp
OUT=gpurun_out/r04v; mkdir -p $OUT
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/debug/host_bound.py 2>&1 | grep "K=100" || exit 1
for i in 1 2; do for ge in 8 1; do
  timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --gather-every $ge > $OUT/b.log 2>&1 || exit $?
  echo "gather_every=$ge K100 $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"])')"
done; done
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-kernel-timer > $OUT/b.log 2>&1 || exit $?
  echo "no-kernel-timer K100 $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"])')"
done
