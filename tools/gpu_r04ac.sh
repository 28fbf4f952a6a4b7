# r04: fps_mid (eager 512 x 2, pipelines 256 x 4) -- GPU tests, then bench lines
export TMPDIR=/tmp
OUT=gpurun_out/r04ac; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do for k in 100 20; do
  w=10; [ $k = 20 ] && w=5
  timeout -k 10 300 python3 bench.py --steps $k --warmup $w --no-cpu-baseline --no-kernel-timer > $OUT/b.log 2>&1 || exit $?
  echo "K$k $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["value_settled"]["value"], d["eager_value"])')"
done; done
