#!/bin/bash
# Round 5: decode GEMMs at the headline batch (M = 1024): gemm_w4 256 x 256 tiles with split-K
# and the parallel combine (every CU busy: o / down 64 tiles x 4 slices) against the tuned
# gemm_xd forms and the library, weights rotated through HBM.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5e; mkdir -p $O
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
{
$P --shape 1024,4096,4096 --rotate 12 --arms lib,x141,v11:4:8,v11:4:-4,v13:4:-4,v11:2:8 &&
$P --shape 1024,4096,4096 --epi residual --rotate 12 --arms x141,v11:4:-4,v13:4:-4 &&
$P --shape 1024,4096,14336 --rotate 4 --arms lib,x242,v11:4:8,v11:4:-4,v13:4:-4,v11:2:-4 &&
$P --shape 1024,6144,4096 --rotate 12 --arms lib,x161,v11:2:8,v11:2:-4,v13:2:-4 &&
$P --shape 1024,28672,4096 --epi silu --rotate 3 --arms v63,v11:2:-4,v13:2:-4
} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | cut -c1-200
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py -k "splitk_timeout or ring or xd_gemm or persistent or splitk" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
