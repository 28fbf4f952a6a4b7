# r04: layer 0 interleaved with layer 1 in the pre-transformed chains (FUSE01, new default) vs
# the separate layer-0 pass (pn2/var/nofuse.so)
export TMPDIR=/tmp
OUT=gpurun_out/r04p; mkdir -p $OUT
V=pointnet-like-pose-estimation_amd/pn2/var
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_full.py tests/test_gpu_sa.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in new old; do
  env=""; [ $v = old ] && env="PN2_TUNING=lib=$V/nofuse.so"
  rm -rf $OUT/prof_$v
  env $env timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timer --no-pipeline > $OUT/prof_$v.log 2>&1 || exit $?
  echo "== $v"; python3 tools/kstats.py $OUT/prof_$v sa_chain | head -3 | tee $OUT/kstats_$v.txt
done
for i in 1 2; do for v in new old; do
  env=""; [ $v = old ] && env="PN2_TUNING=lib=$V/nofuse.so"
  for k in 100 20; do
    w=10; [ $k = 20 ] && w=5
    env $env timeout -k 10 300 python3 bench.py --steps $k --warmup $w --no-cpu-baseline > $OUT/b.log 2>&1 || exit $?
    echo "$v K$k $i $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"])')"
  done
done; done
for c in msg pose; do for v in new old; do
  env=""; [ $v = old ] && env="PN2_TUNING=lib=$V/nofuse.so"
  env $env timeout -k 10 300 python3 bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline > $OUT/b.log 2>&1 || exit $?
  echo "$c $v K100 $(grep '^{' $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"])')"
done; done
