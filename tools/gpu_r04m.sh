# r04: chain ablations (timing only, wrong results): no ring barriers / no hidden epilogues / no
# neighbour-index hop, eager kernel times beside the product build
export TMPDIR=/tmp
OUT=gpurun_out/r04m; mkdir -p $OUT
V=pointnet-like-pose-estimation_amd/pn2/var
for v in base NODMA NOLDS ALL; do
  env=""; [ $v != base ] && env="PN2_TUNING=lib=$V/abl_$v.so"
  rm -rf $OUT/prof_$v
  env $env timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timer --no-pipeline > $OUT/prof_$v.log 2>&1 || exit $?
  echo "== $v"; python3 tools/kstats.py $OUT/prof_$v sa_chain | head -3 | tee $OUT/kstats_$v.txt
done
