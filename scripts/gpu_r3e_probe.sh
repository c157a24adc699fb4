#!/bin/bash
# Round 3: sampler (register top-k path) tests + timing; gemm_w4 at the full decode batch
# (M = 1024) with weights streamed from HBM (--rotate: more weight copies than the MALL
# holds), split-K 1/2/4 against the tuned library.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "sample" > gpurun_out/t_sample.log 2>&1 || { tail -30 gpurun_out/t_sample.log; exit 1; }
tail -1 gpurun_out/t_sample.log
timeout -k 10 200 python -u scripts/sampler_bench.py > gpurun_out/sampler_bench.log 2>&1 || { tail -20 gpurun_out/sampler_bench.log; exit 1; }
grep -v amdgpu gpurun_out/sampler_bench.log
: > gpurun_out/probe_dec_rot.log
for spec in "1024,4096,4096 store 1 10" "1024,4096,4096 store 2 10" "1024,4096,4096 store 4 10" \
            "1024,6144,4096 store 1 8" "1024,6144,4096 store 2 8" \
            "1024,4096,14336 store 1 4" "1024,4096,14336 store 2 4" "1024,4096,14336 store 4 4" \
            "1024,28672,4096 silu 1 2" "1024,128256,4096 store 1 1"; do
  set -- $spec
  timeout -k 10 200 python -u scripts/w4_probe.py --shape $1 --epi $2 --splitk $3 --rotate $4 --group-m 4 --arms lib,v7 --iters 20 >> gpurun_out/probe_dec_rot.log 2>&1 || { tail -5 gpurun_out/probe_dec_rot.log; exit 1; }
done
grep -v amdgpu gpurun_out/probe_dec_rot.log
