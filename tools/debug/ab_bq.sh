# Eager-forward kernel times of the default libpn2 against a variant build (tools/debug/build_var.sh
# <name> ...; PN2_DEBUG_LIB), interleaved twice under rocprofv3 --kernel-trace:
#   VAR=tools/var/<name>.so bash tools/debug/ab_bq.sh      (on the GPU box, from the repo root)
set -u
export TMPDIR=/tmp
VAR=${VAR:?set VAR to a variant .so}
mkdir -p gpurun_out/bqab
for r in 1 2; do
  for v in base var; do
    rm -rf gpurun_out/bqab/kt_$v$r
    if [ $v = var ]; then export PN2_DEBUG_LIB=$VAR; else unset PN2_DEBUG_LIB; fi
    FORWARDS=40 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/bqab/kt_$v$r -o run --output-format csv -- python3 tools/debug/eager_run.py > gpurun_out/bqab/$v$r.log 2>&1 || exit 1
    unset PN2_DEBUG_LIB
    echo "== $v $r: $(grep 'eager forward' gpurun_out/bqab/$v$r.log)"
    python tools/kstats.py gpurun_out/bqab/kt_$v$r | grep -E "ball_query|fps_kernel"
  done
done
