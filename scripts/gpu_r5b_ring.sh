#!/bin/bash
# Round 5: gemm_ring (4-slot LDS ring of 32-deep K stages) - fp32 tests, then interleaved A/B
# against gemm_w4 v63 and hipBLASLt on the four Llama-3-8B prefill shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py -k "ring" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 10 --rounds 5"
{
$P --shape 16384,6144,4096 --arms lib,v63,r4,r8 --group-m 4 &&
$P --shape 16384,4096,4096 --epi residual --arms lib,v63,r4 --group-m 4 &&
$P --shape 16384,28672,4096 --epi silu --arms lib,v63,r8 --group-m 8 &&
$P --shape 16384,4096,14336 --arms lib,v63,r2,r4 --group-m 2
} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | cut -c1-200
