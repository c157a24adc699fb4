#!/bin/bash
# Round 5: kernel-trace anatomy of the Llama-3-70B ask wave at batch 256 on the current tree
# (lm_head on gemm_xd), with the per-pass gap accounting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r5ar
bash scripts/gpu_prof_model.sh r5ar_70b --model llama-3-70b --workload ask --batch 256 --steps 1 --warmup 1 > gpurun_out/r5ar/prof.out 2>&1
rc=$?; tail -3 gpurun_out/r5ar/prof.out; [ $rc -eq 0 ] || exit $rc
mv gpurun_out/r5ar_70b* gpurun_out/r5ar/ 2>/dev/null
grep -B 3 -A 40 '^\*\*prefill' gpurun_out/r5ar/r5ar_70b_summary_full.md | head -80
