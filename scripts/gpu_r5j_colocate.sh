#!/bin/bash
# Round 5: real-size Gemma-2B (smart reply) and Llama-3-8B (summarize) engine groups side by
# side on ONE MI355X with explicit HBM budgets, under concurrent load of both features.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5j; mkdir -p $O
timeout -k 10 500 python -u scripts/colocate_bench.py --smart-mem 0.3 --summary-mem 0.6 \
  --seconds 60 > $O/colocate.json 2> $O/colocate.err || { tail -30 $O/colocate.err; exit 1; }
cat $O/colocate.json
