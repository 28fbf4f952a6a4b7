# r04: the chain ablation builds in the pipeline again, now read on value_settled (the steady
# state after ~80 ms of load) as well as on the contract's first-run value
export TMPDIR=/tmp
OUT=gpurun_out/r04z; mkdir -p $OUT
V=pointnet-like-pose-estimation_amd/pn2/var
for i in 1 2; do for v in base ALL NODMA; do
  env=""; [ $v != base ] && env="PN2_TUNING=lib=$V/abl_$v.so"
  env $env timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-kernel-timer > $OUT/b.log 2>&1 || exit $?
  echo "$v K100 $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["value_settled"]["value"], d["eager_value"])')"
done; done
