#!/bin/bash
# Round-3 GEMM iteration on one MI355X: v7+ numerics, schedule-variant A/B on the prefill
# shapes (qkv / o / gate_up / down of Llama-3-8B at a 16k-token chunk), each at its best
# row-group size (scripts/gpu_w4_groups.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "mfma_gemm" > gpurun_out/t_gemm.log 2>&1 || { tail -20 gpurun_out/t_gemm.log; exit 1; }
tail -2 gpurun_out/t_gemm.log
A=${ARMS:-lib,v7,v8,v9,v10,v11,v12,v13,v14}
: > gpurun_out/probe_var.log
for spec in "16384,6144,4096 store 4" "16384,4096,4096 residual 4" "16384,4096,14336 residual 2" "16384,28672,4096 silu 8"; do
  set -- $spec
  timeout -k 10 300 python -u scripts/w4_probe.py --shape $1 --epi $2 --group-m $3 --arms $A >> gpurun_out/probe_var.log 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/probe_var.log
