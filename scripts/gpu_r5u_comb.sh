#!/bin/bash
# Round 5: gemm_xd split-K combine with batched slab loads (one latency per fragment group, not
# per fragment) and stream-K forms (splitk digit 0): fp32-reference tests of every xd form /
# epilogue, then the decode shapes (2x8 split / stream-K forms vs the tuned forms).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_gpu.py tests/test_kernels_gpu.py -k "xd or splitk or moe or stream" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
{
$P --shape 1024,4096,4096 --rotate 12 --arms lib,x141,x284,x280,x1280,x240,x140,x242 &&
$P --shape 1024,4096,4096 --epi residual --rotate 12 --arms x141,x284,x280,x240 &&
$P --shape 1024,4096,14336 --rotate 4 --arms lib,x242,x284,x280,x1280,x240 &&
$P --shape 1024,6144,4096 --rotate 12 --arms lib,x161,x282,x280,x1280,x240,x160 &&
$P --shape 1024,28672,4096 --epi silu --rotate 3 --arms v63,x281,x280,x1280,x240 &&
$P --shape 256,10240,8192 --rotate 3 --arms lib,x243,x244,x280,x1280,x240,x1240 &&
$P --shape 256,8192,28672 --rotate 2 --arms lib,x244,x1244,x280,x1280,x240,x1240 &&
$P --shape 256,57344,8192 --epi silu --rotate 2 --arms v63,x281,x1281,x280,x1280
} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | cut -c1-170
