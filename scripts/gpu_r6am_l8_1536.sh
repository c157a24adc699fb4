#!/bin/bash
# Round 6: Llama-3-8B decode at batch 1536 (above the decode buckets): library vs gemm_xd /
# gemm_w4 forms for qkv / o / down / gate_up+GLU, interleaved per shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6am; mkdir -p $O
p() {  # tag shape epi arms
  timeout -k 10 240 python -u scripts/w4_probe.py --shape $2 --epi $3 --arms $4 --iters 10 --rounds 5 > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
  grep -v amdgpu $O/$1.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('$1', d['arm'], d['us_med'])"
}
p qkv 1536,6144,4096 store lib,x141,x241,x242,x281,x1241,v63:1:8,v63:1:4
p o 1536,4096,4096 store lib,x141,x142,x241,x242,x243,v63:1:8
p down 1536,4096,14336 store lib,x142,x242,x243,x244,x282,x1242
p gu 1536,28672,4096 silu lib,x141,x241,x281,v63:1:4,v63:1:8
