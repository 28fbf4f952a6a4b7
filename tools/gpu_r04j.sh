# r04: v_permlane32_swap half-column max (new) vs ds_bpermute (old build pn2/var/permold.so)
export TMPDIR=/tmp
OUT=gpurun_out/r04j; mkdir -p $OUT
V=pointnet-like-pose-estimation_amd/pn2/var
timeout -k 10 500 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_full.py tests/test_gpu_sa.py tests/test_gpu_configs.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in new old; do
  env=""; [ $v = old ] && env="PN2_TUNING=lib=$V/permold.so"
  rm -rf $OUT/prof_$v
  env $env timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timer --no-pipeline > $OUT/prof_$v.log 2>&1 || exit $?
  echo "== $v"; python3 tools/kstats.py $OUT/prof_$v pn2:: | head -8 | tee $OUT/kstats_$v.txt
done
for i in 1 2; do for v in new old; do
  env=""; [ $v = old ] && env="PN2_TUNING=lib=$V/permold.so"
  env $env timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench_$v$i.log 2>&1 || exit $?
  echo "$v K100 $i $(grep '^{' $OUT/bench_$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"], d["roofline"]["frac"])')"
  env $env timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench20_$v$i.log 2>&1 || exit $?
  echo "$v K20 $i $(grep '^{' $OUT/bench20_$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"])')"
done; done
