#!/bin/bash
# Round 3 final (persistent gemm_w4 by default): kernel-trace profile of the headline on the final tree (per-phase kernel
# anatomy + idle accounting of the timed step), then the whole GPU suite and smoke().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_prof_model.sh r3t --steps 2 --warmup 1 > gpurun_out/prof_r3t.out 2>&1
rc=$?; tail -3 gpurun_out/prof_r3t.out; [ $rc -eq 0 ] || exit $rc
python scripts/trace_gaps.py gpurun_out/r3t_kernel_trace.csv.gz > gpurun_out/r3t_gaps.txt 2>&1 || true
head -3 gpurun_out/r3t_gaps.txt
rm -f gpurun_out/r3t_kernel_trace.csv.gz.keep
bash scripts/gpu_r3d_verify.sh
