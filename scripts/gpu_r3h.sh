#!/bin/bash
# Round 3: sampler tail (rank-count sort + one block scan) tests + timing, then the
# medium-M GEMM tuning at the 160-256-row decode buckets (scripts/gpu_r3f_midm256.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k "sample" > gpurun_out/t_sample.log 2>&1 || { tail -30 gpurun_out/t_sample.log; exit 1; }
tail -1 gpurun_out/t_sample.log
timeout -k 10 200 python -u scripts/sampler_bench.py --rounds 3 > gpurun_out/sampler_bench.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/sampler_bench.log
bash scripts/gpu_r3f_midm256.sh
