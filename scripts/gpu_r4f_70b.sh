#!/bin/bash
# Round 4: Llama-3-70B decode projections at the 192 / 256 buckets on gemm_w4 (split-K in the
# K-slice-by-XCD order; persistent GLU for gate_up) against the tuned library, weights
# streamed from HBM.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r4f
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4f
: > $O/probe.log
for M in 256 192; do
for spec in "$M,8192,28672 store 2 lib,v7:8:-1,v11:8:-1,v11:8:1,v11:4:-2" \
            "$M,8192,8192 store 4 lib,v7:8:-1,v11:8:-1,v11:4:-2" \
            "$M,10240,8192 store 3 lib,v11:4:-2,v11:4:2" \
            "$M,57344,8192 silu 1 lib,v15:1:8,v7:1:8"; do
  set -- $spec
  timeout -k 10 200 python -u scripts/w4_probe.py --shape $1 --epi $2 --rotate $3 --arms $4 --iters 10 >> $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
done
done
for spec in "1024,4096,4096 store 10 lib,v11:4:-4,v11:4:4,v11:2:-2" \
            "1024,4096,14336 store 4 lib,v11:4:-4,v11:4:4,v11:2:-2" \
            "768,4096,14336 store 4 lib,v11:4:-4,v11:4:4" \
            "512,4096,14336 store 4 lib,v11:8:-2,v11:4:-2"; do
  set -- $spec
  timeout -k 10 200 python -u scripts/w4_probe.py --shape $1 --epi $2 --rotate $3 --arms $4 --iters 10 >> $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
done
grep -v amdgpu $O/probe.log
