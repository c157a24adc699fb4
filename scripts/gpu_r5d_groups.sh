#!/bin/bash
# Round 5: gemm_w4 v63 tile-order row groups on the Llama-3-8B prefill shapes (the r5c PMC
# shows v63 on down at group 2 with 46 % more L2 misses than hipBLASLt: 2 x 16 tile blocks per
# XCD need 18 operand panels per K step, 4 x 8 blocks need 12).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5d; mkdir -p $O
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 10 --rounds 5"
{
$P --shape 16384,4096,14336 --arms lib,v63:1:2,v63:1:4,v63:1:8,v63:1:16 &&
$P --shape 16384,6144,4096 --arms lib,v63:1:2,v63:1:4,v63:1:8 &&
$P --shape 16384,4096,4096 --epi residual --arms lib,v63:1:2,v63:1:4,v63:1:8 &&
$P --shape 16384,28672,4096 --epi silu --arms v63:1:4,v63:1:8,v63:1:16
} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | cut -c1-200
