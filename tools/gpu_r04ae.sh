# r04: eager launch profile (dense_lds for wide layers, 16-wave ball query, 8x2 FPS) with the
# pipelines under PIPELINE_PROFILE -- GPU tests, SSG bench, every config
export TMPDIR=/tmp
OUT=gpurun_out/r04ae; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do for k in 100 20; do
  w=10; [ $k = 20 ] && w=5
  timeout -k 10 300 python3 bench.py --steps $k --warmup $w --no-cpu-baseline > $OUT/b.log 2>&1 || exit $?
  echo "ssg K$k $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["value_settled"]["value"], d["eager_value"], d["roofline"]["frac"])')"
done; done
for c in msg pose stress v1; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $OUT/$c.log 2>&1 || { tail -5 $OUT/$c.log; exit 1; }
  grep '^{' $OUT/$c.log | tail -1 > $OUT/$c.json
  echo "$c $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], (d.get("value_settled") or {}).get("value"), d["eager_value"], (d.get("roofline") or {}).get("frac"))' $OUT/$c.json)"
done
