#!/bin/bash
# Round 5: lm_head (vocabulary-wide projection) on gemm_xd forms vs the tuned library, every
# decode bucket (a first pass at M = 1024 / 896 / 512 / 256 / 224: profiles/r5ak/tune_first.log).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5ak; mkdir -p $O
timeout -k 10 600 python -u scripts/tune_xd.py --configs llama-3-8b:1,llama-3-70b:1,gemma-2b:1,mixtral-8x7b:1 --gemms lm_head --min-gain 0 --nt-any --out $O/xd_lmhead.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
cat $O/tune.log
