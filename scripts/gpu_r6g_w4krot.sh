#!/bin/bash
# Round 6: long-K gemm_w4 tile-order / K-rotation sweep against hipBLASLt (prefill down shapes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 400 python -u scripts/w4_probe.py --shape 16384,4096,14336 --epi residual --arms lib,v63:1:4,v63:1:4:k4,v63:1:4:k2,v63:1:4:k1,v47:1:4,v63:1:8:k4,v63:1:2:k4,v7:1:4,v7:1:8 --iters 8 --rounds 5 > $O/down8b.log 2>&1 || { tail -20 $O/down8b.log; exit 1; }
grep -v amdgpu $O/down8b.log | cut -c1-200
timeout -k 10 500 python -u scripts/w4_probe.py --shape 16384,8192,28672 --epi residual --arms lib,v63:1:4,v63:1:4:k4,v63:1:4:k1,v47:1:4,v7:1:4,v7:1:8,v7:1:2 --iters 3 --rounds 4 > $O/down70b.log 2>&1 || { tail -20 $O/down70b.log; exit 1; }
grep -v amdgpu $O/down70b.log | cut -c1-200
