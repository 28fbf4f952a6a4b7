# r04: full GPU suite, then the SQ MFMA pass of every config (profiles/sq_mfma.json)
export TMPDIR=/tmp
OUT=gpurun_out/r04i; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="ssg msg pose stress v1" bash tools/sq_mfma.sh > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
grep -A3 "kernel" $OUT/sq.log | cut -c1-200 | head -40
