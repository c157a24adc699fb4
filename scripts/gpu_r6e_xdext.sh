#!/bin/bash
# Round 6: extended gemm_xd form search (every tile x split-K 1..8, plain + nt) against today's
# tuned route, for the 70B ask decode (192-256 rows) and the 8B headline decode (896 / 1024).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 900 python -u scripts/tune_xd_ext.py --configs llama-3-70b:1 --ms 192,224,256,320 --out $O/xd_ext_70b.json > $O/tune70.log 2>&1 || { tail -20 $O/tune70.log; exit 1; }
grep -v FAILED $O/tune70.log | grep -v amdgpu
timeout -k 10 600 python -u scripts/tune_xd_ext.py --configs llama-3-8b:1 --ms 768,896,1024 --out $O/xd_ext_8b.json > $O/tune8.log 2>&1 || { tail -20 $O/tune8.log; exit 1; }
grep -v FAILED $O/tune8.log | grep -v amdgpu
grep -c FAILED $O/tune70.log $O/tune8.log || true
