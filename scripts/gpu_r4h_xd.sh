#!/bin/bash
# Round 4: gemm_xd LDS ring depth A/B (S - 1 K tiles in flight per CU) at the decode shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4h
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py -k "xd" > gpurun_out/r4h/tests.log 2>&1 || { tail -30 gpurun_out/r4h/tests.log; exit 1; }
tail -2 gpurun_out/r4h/tests.log
P="timeout -k 10 120 python -u scripts/w4_probe.py --iters 20 --rounds 7"
{
$P --shape 1024,4096,4096 --arms lib,x4:4,x4:5 --rotate 10 &&
$P --shape 1024,6144,4096 --arms lib,x6:3,x6:4 --rotate 8 &&
$P --shape 1024,4096,14336 --arms lib,x4:4,x4:5 --rotate 4 &&
$P --shape 512,4096,4096 --arms lib,x2:4,x2:6 --rotate 10 &&
$P --shape 512,4096,14336 --arms lib,x2:4,x2:6 --rotate 4 &&
$P --shape 512,6144,4096 --arms lib,x2:4,x2:6 --rotate 8 &&
$P --shape 768,4096,4096 --arms lib,x4:5,x2:6 --rotate 10 &&
$P --shape 768,6144,4096 --arms lib,x6:4,x4:5,x2:6 --rotate 8 &&
$P --shape 768,4096,14336 --arms lib,x4:5,x2:6 --rotate 4
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4h/probe.log
