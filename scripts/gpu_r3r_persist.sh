#!/bin/bash
# Round 3: persistent gemm_w4 (variant 15, cross-tile DMA prefetch) - numerics, then the
# prefill projection shapes against the per-tile form (variant 7) and hipBLASLt.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r3r
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -q --timeout 200 --timeout-method thread -k "w4 or matches_fp32" > gpurun_out/r3r/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3r/tests.log; [ $rc -eq 0 ] || exit $rc
for sh in "16384,6144,4096 store 4" "16384,4096,4096 residual 4" "16384,28672,4096 silu 8" "16384,4096,14336 residual 2" "4400,28672,4096 silu 8" "1024,28672,4096 silu 8"; do
  set -- $sh
  timeout -k 10 120 python -u scripts/w4_probe.py --shape $1 --epi $2 --group-m $3 --arms lib,v7,v15 --iters 10 --rounds 5 >> gpurun_out/r3r/probe.log 2>&1 || exit 1
done
cat gpurun_out/r3r/probe.log
