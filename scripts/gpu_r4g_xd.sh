#!/bin/bash
# Round 4: gemm_xd (XCD-partitioned 128-row decode GEMM) - fp32 tests, then A/B against the
# tuned library at the Llama-3-8B decode shapes (weights rotated: streamed from HBM).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4g
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py -k "xd" > gpurun_out/r4g/tests.log 2>&1 || { tail -30 gpurun_out/r4g/tests.log; exit 1; }
tail -2 gpurun_out/r4g/tests.log
P="timeout -k 10 120 python -u scripts/w4_probe.py --iters 20 --rounds 5"
{
$P --shape 1024,4096,4096 --arms lib,x4,x2 --rotate 10 &&
$P --shape 1024,6144,4096 --arms lib,x6,x4,x2 --rotate 8 &&
$P --shape 1024,4096,14336 --arms lib,x4,x2 --rotate 4 &&
$P --shape 896,4096,4096 --arms lib,x4,x2 --rotate 10 &&
$P --shape 768,4096,4096 --arms lib,x4,x2 --rotate 10 &&
$P --shape 512,4096,4096 --arms lib,x4,x2 --rotate 10 &&
$P --shape 512,4096,14336 --arms lib,x4,x2 --rotate 4 &&
$P --shape 512,6144,4096 --arms lib,x6,x2 --rotate 8 &&
$P --shape 1024,128256,4096 --arms lib,x4,x6 --rotate 1
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4g/probe.log
