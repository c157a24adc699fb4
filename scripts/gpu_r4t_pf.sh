#!/bin/bash
# Round 4: gemm_xd weight-prefetch forms (form + 1000): fp32 tests, then interleaved A/B on
# the weight-streaming shapes (Llama-3-70B at M = 192-256, Llama-3-8B at 256-1024).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4t
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py -k "xd" > gpurun_out/r4t/tests.log 2>&1 || { tail -30 gpurun_out/r4t/tests.log; exit 1; }
tail -1 gpurun_out/r4t/tests.log
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
{
$P --shape 256,8192,28672 --arms lib,x244,x1244,x1243 --rotate 2 &&
$P --shape 256,8192,8192 --arms lib,x121,x1121,x1242 --rotate 4 &&
$P --shape 256,10240,8192 --arms lib,x243,x1243,x1121 --rotate 4 &&
$P --shape 256,57344,8192 --epi silu --arms lib,x241,x1241 --rotate 2 &&
$P --shape 192,8192,28672 --arms lib,x244,x1244 --rotate 2 &&
$P --shape 1024,4096,14336 --arms lib,x242,x1242 --rotate 4 &&
$P --shape 1024,4096,4096 --arms lib,x141,x1141 --rotate 10 &&
$P --shape 512,4096,14336 --arms lib,x242,x1242,x1121 --rotate 4 &&
$P --shape 256,4096,14336 --arms lib,x244,x1244 --rotate 4
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4t/probe.log
