#!/bin/bash
# Round 5: the prefill down projection (the library kernel left in 8B / 70B prefill): gemm_w4
# store vs residual epilogue vs the library, persistent (v63) and non-persistent (v7) schedules,
# row-group 4 / 8 / 16, interleaved in one process per shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5ao; mkdir -p $O
for epi in store residual; do
  timeout -k 10 300 python -u scripts/w4_probe.py --shape 16384,4096,14336 --epi $epi --arms lib,v63,v7,v63:1:4,v63:1:16 --rotate 2 --iters 6 >> $O/down8b.log 2>&1 || { tail -5 $O/down8b.log; exit 1; }
done
timeout -k 10 300 python -u scripts/w4_probe.py --shape 16384,8192,28672 --epi residual --arms lib,v63,v7 --rotate 2 --iters 4 --rounds 3 >> $O/down70b.log 2>&1 || { tail -5 $O/down70b.log; exit 1; }
grep -h '"arm"' $O/down8b.log $O/down70b.log | cut -c1-200
