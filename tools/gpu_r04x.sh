# r04: grid ball query v2 -- per-launch times, parity, bench
export TMPDIR=/tmp
OUT=gpurun_out/r04x; mkdir -p $OUT
timeout -k 10 120 python tools/debug/bq_grid_time.py 2>&1 | grep us/launch || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bq_grid.py tests/test_gpu_large_k.py tests/test_gpu_ops.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for m in 0 1; do
  PN2_TUNING=bq_grid=$m timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b$m.log 2>&1 || exit $?
  echo "bq_grid=$m $(grep '^{' $OUT/b$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["value_settled"]["value"], d["eager_value"], {k: v for k, v in d["kernels"].items() if "ball" in k})')"
done
