# r04: what bounds the pipelined steady state -- graph node counts per batch, and the kernel
# timeline's busy fraction over the last 20 ms of three K = 100 runs
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04y; mkdir -p $OUT
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python tools/debug/graph_nodes.py > $OUT/nodes.txt 2>&1 || { cat $OUT/nodes.txt; exit 1; }
cat $OUT/nodes.txt
cd /tmp && GPU_MAX_HW_QUEUES=8 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $GRAFT_REPO_ROOT/tools/debug/bench_gap.py bare > $OUT/kt.log 2>&1 || { tail $OUT/kt.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/debug/busy_union.py $(find $OUT/kt -name "*kernel_trace.csv" | head -1) 20
