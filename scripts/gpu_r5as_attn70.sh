#!/bin/bash
# Round 5: decode attention at the 70B ask shapes (Hq 64, Hkv 8): partition sweep of variant 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5as; mkdir -p $O
timeout -k 10 300 python -u scripts/decode_attn_bench.py 3,1 llama70b > $O/attn70.log 2>&1 || { tail -20 $O/attn70.log; exit 1; }
grep -v amdgpu $O/attn70.log
