set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ta
export TMPDIR=/tmp
CMD="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timer --no-pipeline"
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE -d gpurun_out/ta/p1 -o run --output-format csv -- $CMD > gpurun_out/ta/p1.log 2>&1 || { echo p1 fail; tail -3 gpurun_out/ta/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TD_BUSY_avr TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d gpurun_out/ta/p2 -o run --output-format csv -- $CMD > gpurun_out/ta/p2.log 2>&1 || { echo p2 fail; tail -3 gpurun_out/ta/p2.log; exit 1; }
echo ok
