#!/bin/bash
# Round 3: where the split-K partial-plane decode form loses (GEMM vs norm halves, real
# shapes, HBM-streamed weights); sampler with the unrolled rank count; medium-M GEMM tuning
# at the 160-256-row decode buckets.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/partials_probe.py > gpurun_out/partials_probe.log 2>&1 || { tail -20 gpurun_out/partials_probe.log; exit 1; }
grep -v amdgpu gpurun_out/partials_probe.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k "sample" > gpurun_out/t_sample.log 2>&1 || { tail -30 gpurun_out/t_sample.log; exit 1; }
tail -1 gpurun_out/t_sample.log
timeout -k 10 200 python -u scripts/sampler_bench.py --rounds 3 > gpurun_out/sampler_bench.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/sampler_bench.log | grep randn_s2
bash scripts/gpu_r3f_midm256.sh
