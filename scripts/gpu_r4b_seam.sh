#!/bin/bash
# Round 4: prefill-shape gemm_w4, persistent (v15) vs persistent with a per-XCD K rotation
# (v31: the eight XCDs reach their tile seams at different times) vs hipBLASLt; and a K
# sweep at fixed M x N to separate the per-tile cost from the K-loop rate.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r4b
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4b
: > $O/probe.log
for spec in "16384,4096,2048 store 2 lib,v15:1:4,v31:1:4" \
            "16384,4096,4096 store 2 lib,v15:1:4,v31:1:4" \
            "16384,4096,8192 store 2 lib,v15:1:4,v31:1:4" \
            "16384,4096,14336 store 2 lib,v15:1:2,v31:1:2" \
            "16384,6144,4096 store 2 lib,v15:1:4,v31:1:4" \
            "16384,4096,4096 residual 2 lib,v15:1:4,v31:1:4" \
            "16384,28672,4096 silu 2 lib,v15:1:8,v31:1:8" \
            "16384,4096,14336 residual 2 lib,v15:1:2,v31:1:2" \
            "1024,28672,4096 silu 2 lib,v15:1:8,v31:1:8" \
            "1024,128256,4096 store 1 lib,v15:1:4,v31:1:4"; do
  set -- $spec
  timeout -k 10 200 python -u scripts/w4_probe.py --shape $1 --epi $2 --rotate $3 --arms $4 --iters 10 >> $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
done
grep -v amdgpu $O/probe.log
