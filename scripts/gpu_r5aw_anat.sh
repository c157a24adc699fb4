#!/bin/bash
# Round 5: kernel-trace anatomy of the headline (Llama-3-8B smart reply, batch 1024) on the last
# tree, with the gap accounting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r5aw
bash scripts/gpu_prof_model.sh r5aw --steps 2 --warmup 1 > gpurun_out/r5aw/prof.out 2>&1
rc=$?; tail -3 gpurun_out/r5aw/prof.out; [ $rc -eq 0 ] || exit $rc
mv gpurun_out/r5aw.* gpurun_out/r5aw_* gpurun_out/r5aw/ 2>/dev/null
python scripts/trace_gaps.py gpurun_out/r5aw/r5aw_kernel_trace.csv.gz > gpurun_out/r5aw/gaps.txt 2>&1
head -4 gpurun_out/r5aw/r5aw_summary_full.md; head -3 gpurun_out/r5aw/gaps.txt
