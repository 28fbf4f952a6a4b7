# r04: culled FPS coalesced pass A (tests + traffic), SQ counter passes of the current chains
export TMPDIR=/tmp
OUT=gpurun_out/r04h; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fps_cull.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for P in FETCH_SIZE WRITE_SIZE; do
  rm -rf $OUT/pmc_$P
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/pmc_$P -o run --output-format csv -- python3 tools/debug/fps_one.py 128 16384 512 102444 > $OUT/pmc_$P.log 2>&1 || exit $?
  grep -h fps_cull $OUT/pmc_$P/*counter_collection.csv | head -2 | cut -c1-40,200-400
done
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
bash tools/sq_pmc.sh > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
cp gpurun_out/sqpmc/summary.txt $OUT/sq_summary.txt
head -30 $OUT/sq_summary.txt | cut -c1-250
