# r04 final: every BASELINE config's bench line with the final build
export TMPDIR=/tmp
OUT=gpurun_out/r04ag; mkdir -p $OUT
for c in msg pose stress v1; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $OUT/$c.log 2>&1 || { tail -5 $OUT/$c.log; exit 1; }
  grep '^{' $OUT/$c.log | tail -1 > $OUT/$c.json
  echo "$c $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], (d.get("value_settled") or {}).get("value"), d["eager_value"], (d.get("roofline") or {}).get("frac"))' $OUT/$c.json)"
done
