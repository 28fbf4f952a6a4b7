export TMPDIR=/tmp
OUT=gpurun_out/r04c; mkdir -p $OUT
PN2_TUNING=lib=pointnet-like-pose-estimation_amd/pn2/var/fpsstats.so timeout -k 10 120 python -u tools/debug/fps_cull_stats.py stats > $OUT/fpsstats.txt 2>&1
PN2_TUNING=lib=pointnet-like-pose-estimation_amd/pn2/var/fpsfloor.so timeout -k 10 120 python -u tools/debug/fps_cull_stats.py time >> $OUT/fpsstats.txt 2>&1
cat $OUT/fpsstats.txt | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_full.py tests/test_gpu_configs.py tests/test_gpu_bf16.py tests/test_gpu_large_k.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in persist nopersist; do
  env=""; [ $v = nopersist ] && env="PN2_TUNING=chain_persist=0"
  rm -rf $OUT/prof_$v
  env $env timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timer --no-pipeline > $OUT/prof_$v.log 2>&1 || exit $?
  echo "== $v"; python3 tools/kstats.py $OUT/prof_$v sa_chain | tee $OUT/kstats_$v.txt
done
for i in 1 2; do for v in persist nopersist; do
  env=""; [ $v = nopersist ] && env="PN2_TUNING=chain_persist=0"
  env $env timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench_$v$i.log 2>&1 || exit $?
  echo "$v $i $(grep '^{' $OUT/bench_$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"], d["roofline"]["frac"])')"
done; done
