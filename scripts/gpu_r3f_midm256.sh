#!/bin/bash
# Round 3: medium-M decode GEMM extended to 129-256 rows (one workgroup per CU, AGPR
# accumulators): numerics, then the per-shape tuning against the engine's library path
# for Llama-3-70B (TP 1) and Llama-3-8B at the 160-256 decode buckets (W streamed from HBM).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "midm" > gpurun_out/t_midm.log 2>&1 || { tail -30 gpurun_out/t_midm.log; exit 1; }
tail -1 gpurun_out/t_midm.log
timeout -k 10 900 python -u scripts/tune_midm.py --configs llama-3-70b:1,llama-3-8b:1 --ms 160,192,224,256 --out gpurun_out/midm256_tuned.json > gpurun_out/tune_midm256.log 2>&1 || { tail -20 gpurun_out/tune_midm256.log; exit 1; }
grep -v amdgpu gpurun_out/tune_midm256.log
