#!/bin/bash
# Round 6: Gemma-2B decode at its 2,048-row batch (beyond the tuned decode buckets): the library
# GEMMs of the decode pass against gemm_xd / gemm_w4 forms, interleaved per shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6ak; mkdir -p $O
p() {  # tag shape epi arms
  timeout -k 10 240 python -u scripts/w4_probe.py --shape $2 --epi $3 --arms $4 --iters 10 --rounds 5 > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
  grep -v amdgpu $O/$1.log | tail -14
}
p qkv 2048,2560,2048 store lib,x121,x122,x141,x142,x241,x242,x1241,v63:1:8,v63:1:4
p o 2048,2048,2048 residual lib,x121,x122,x141,x142,x241,x242,x1242,v63:1:8
p down 2048,2048,16384 residual lib,x122,x124,x142,x144,x242,x244,x282,x1244,v7:2:8,v7:4:8
p lmhead 2048,256000,2048 store lib,x241,x281,x1281,v63:1:8,v63:1:4
