#!/bin/bash
# Round 5: RMSNorm with non-temporal stores vs plain (graph-replayed decode-sized norms), then
# the 70B ask wave at batch 256 with each form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5ax; mkdir -p $O
timeout -k 10 300 python -u scripts/norm_probe.py --graph > $O/norm.log 2>&1 || { tail -20 $O/norm.log; exit 1; }
grep -v amdgpu $O/norm.log
