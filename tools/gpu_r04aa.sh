# r04: cold vs warm host issue; every BASELINE config's bench line at round end
export TMPDIR=/tmp
OUT=gpurun_out/r04aa; mkdir -p $OUT
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python tools/debug/cold_host.py 2>&1 | grep -v amdgpu.ids || exit 1
for c in msg pose stress v1; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $OUT/$c.log 2>&1 || { tail -5 $OUT/$c.log; exit 1; }
  grep '^{' $OUT/$c.log | tail -1 > $OUT/$c.json
  echo "$c $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"], (d.get("value_settled") or {}).get("value"), d["eager_value"], (d.get("roofline") or {}).get("frac"))' $OUT/$c.json)"
done
