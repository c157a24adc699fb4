#!/bin/bash
# Round 5: gemm_w4 fixed cost per tile (prologue / epilogue / seam) vs main-loop cost: the
# same prefill shapes at K = 2048 / 4096 / 8192 (time = tiles x (c0 + c1 x K tiles)).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5q; mkdir -p $O
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 10 --rounds 5"
{
for k in 2048 4096 8192; do
  $P --shape 16384,28672,$k --epi silu --arms lib,v63:1:4 || exit 1
  $P --shape 16384,6144,$k --arms lib,v63:1:8 || exit 1
done
} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | cut -c1-200
