# r04 round end, part 2: PMC traffic of every config, the SQ MFMA pass of every config, the K = 20
# timeline
export TMPDIR=/tmp
STEPS=pmc PMC_CONFIGS="ssg msg pose stress" bash tools/gpu_check.sh > gpurun_out/pmc_all.log 2>&1 || { tail -5 gpurun_out/pmc_all.log; exit 1; }
grep -h "per_call" gpurun_out/pmc_summary_*.txt
CONFIGS="ssg msg pose stress v1" bash tools/sq_mfma.sh > gpurun_out/sq_all.log 2>&1 || { tail -5 gpurun_out/sq_all.log; exit 1; }
mkdir -p gpurun_out/end
GPU_MAX_HW_QUEUES=8 FROM_START=1 K=20 timeout -k 10 120 python tools/debug/gpipe_events.py > gpurun_out/end/timeline_k20.txt 2>&1 || exit 1
head -4 gpurun_out/end/timeline_k20.txt
