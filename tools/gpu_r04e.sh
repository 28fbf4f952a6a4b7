# r04: culled FPS v2, chain prologue reorder + pool atomics + asm weight reads (A/B vs HEAD build)
export TMPDIR=/tmp
OUT=gpurun_out/r04e; mkdir -p $OUT
V=pointnet-like-pose-estimation_amd/pn2/var
timeout -k 10 500 python -u -m pytest tests/test_gpu_fps_cull.py tests/test_gpu_mlp.py tests/test_gpu_full.py tests/test_gpu_sa.py tests/test_gpu_configs.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in new asmr0 old; do
  env=""; [ $v = old ] && env="PN2_TUNING=lib=$V/chainold.so"; [ $v = asmr0 ] && env="PN2_TUNING=lib=$V/asmr0.so"
  rm -rf $OUT/prof_$v
  env $env timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timer --no-pipeline > $OUT/prof_$v.log 2>&1 || exit $?
  echo "== $v"; python3 tools/kstats.py $OUT/prof_$v sa_chain | tee $OUT/kstats_$v.txt
done
for i in 1 2; do for v in new asmr0 old; do
  env=""; [ $v = old ] && env="PN2_TUNING=lib=$V/chainold.so"; [ $v = asmr0 ] && env="PN2_TUNING=lib=$V/asmr0.so"
  env $env timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench_$v$i.log 2>&1 || exit $?
  echo "$v $i $(grep '^{' $OUT/bench_$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["eager_value"], d["roofline"]["frac"])')"
done; done
timeout -k 10 300 python -u tools/bench_fps.py --cull=0,1,25612,25622,102422,102414,102424,102442,102444,102482 --tag cull2 > $OUT/fps.log 2>&1 || exit $?
grep -v amdgpu $OUT/fps.log | cut -c1-110
