#!/bin/bash
# Round 5: per-iteration rate of gemm_xd's 256 x 256 tile (2x8, two 64 KiB LDS stages) at the
# 8B decode shapes (M = 1024): one round of 64 work items (x281 on o: no CU contention) vs the
# full chip (split-K 4 = 256 items), against the tuned forms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5t; mkdir -p $O
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
{
$P --shape 1024,4096,4096 --rotate 12 --arms lib,x141,x281,x282,x284,x1281,x1284,x242,x244 &&
$P --shape 1024,4096,14336 --rotate 4 --arms lib,x242,x281,x282,x284,x1284,x244 &&
$P --shape 1024,6144,4096 --rotate 12 --arms lib,x161,x281,x282,x283,x1282,x243 &&
$P --shape 1024,28672,4096 --epi silu --rotate 3 --arms v63,x281,x1281,x282,x241
} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | cut -c1-200
