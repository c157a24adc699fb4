#!/bin/bash
# gemm_w4 at the full decode batch (Llama-3-8B, M = 1024): reduce-scatter split-K (v11) vs the
# last-arriver combine (v7) vs the library.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "mfma_gemm or reduce_scatter" > gpurun_out/t_gemm.log 2>&1 || { tail -30 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
: > gpurun_out/probe_dec.log
for spec in "1024,4096,4096 residual 4" "1024,4096,14336 residual 4" "1024,6144,4096 store 2" "1024,4096,4096 residual 2" "1024,4096,14336 residual 2"; do
  set -- $spec
  timeout -k 10 200 python -u scripts/w4_probe.py --shape $1 --epi $2 --splitk $3 --group-m 4 --arms lib,v7,v11 --iters 20 | sed "s/}/, \"sk\": $3}/" >> gpurun_out/probe_dec.log 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/probe_dec.log
