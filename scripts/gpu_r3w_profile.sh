#!/bin/bash
# Round 3, last tree: kernel-trace anatomy of the headline (persistent gemm_w4, two-workgroup
# sampler, lazy request events) + idle accounting of the timed step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_prof_model.sh r3w --steps 2 --warmup 1 > gpurun_out/prof_r3w.out 2>&1
rc=$?; tail -3 gpurun_out/prof_r3w.out; [ $rc -eq 0 ] || exit $rc
python scripts/trace_gaps.py gpurun_out/r3w_kernel_trace.csv.gz > gpurun_out/r3w_gaps.txt 2>&1 || true
head -8 gpurun_out/r3w_gaps.txt
cut -c1-300 gpurun_out/r3w.json
