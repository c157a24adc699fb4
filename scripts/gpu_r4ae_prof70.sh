#!/bin/bash
# Round 4: kernel-trace anatomy of the Llama-3-70B ask wave at batch 256 (one GPU) with the
# non-temporal gemm_xd forms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_prof_model.sh r4ae_70b --model llama-3-70b --workload ask --batch 256 --steps 1 --warmup 1 > gpurun_out/prof_r4ae.out 2>&1
rc=$?; tail -3 gpurun_out/prof_r4ae.out; [ $rc -eq 0 ] || exit $rc
head -60 gpurun_out/r4ae_70b_summary.md
