#!/bin/bash
# Round 5: gemm_xd 256 x 256 tile with split LDS rings (2 A + 3 B stages of 32 KiB: two weight
# K tiles in flight instead of one): fp32 tests of every xd / grouped-MoE form, then the 2x8
# forms against the tuned forms at the 8B (M = 1024) and 70B (M = 256) decode shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_gpu.py tests/test_kernels_gpu.py -k "xd or splitk or moe" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
{
$P --shape 1024,28672,4096 --epi silu --rotate 3 --arms v63,x281,x1281,x241 &&
$P --shape 256,57344,8192 --epi silu --rotate 2 --arms v63,x1281,x281,x1241 &&
$P --shape 1024,4096,4096 --rotate 12 --arms x141,x281,x282,x284,x242 &&
$P --shape 1024,4096,14336 --rotate 4 --arms x242,x282,x284,x1284 &&
$P --shape 1024,6144,4096 --rotate 12 --arms x161,x281,x282,x283 &&
$P --shape 256,10240,8192 --rotate 3 --arms x1243,x1282,x1283,x1284 &&
$P --shape 256,8192,8192 --rotate 3 --arms x1244,x1282,x1284 &&
$P --shape 256,8192,28672 --rotate 2 --arms x1244,x1282,x1284
} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | python3 -c "import sys,json;[print(json.loads(l)['shape'],json.loads(l)['epi'],json.loads(l)['arm'],json.loads(l)['us_med'],json.loads(l)['err']) for l in sys.stdin]"
