# r04: eager launch-choice A/B (SSG in-process, interleaved), then the other configs' eager
# forward with dense_lds=1,bq_waves=16 vs default
export TMPDIR=/tmp
OUT=gpurun_out/r04ad; mkdir -p $OUT
EAGER_AB_SET=short timeout -k 10 300 python tools/debug/eager_ab.py 3 2>&1 | grep "clouds/s\|differs" || exit 1
for c in msg pose stress v1; do for v in def new; do
  env=""; [ $v = new ] && env="PN2_TUNING=dense_lds=1,bq_waves=16"
  env $env timeout -k 10 300 python3 bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timer > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
  echo "$c $v $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], (d.get("value_settled") or {}).get("value"), d["eager_value"])')"
done; done
