#!/bin/bash
# Round 5: MoE variant 3 defaults on Mixtral shapes + a kernel trace of the T = 1024 layer.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r5l; mkdir -p $O
true

cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o moe -- python3 $R/scripts/moe_bench.py 14336 1024 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' | head -1 | xargs head -12 | cut -c1-200
