#!/bin/bash
# Round 5: re-measure BASELINE rows on the current tree (one timed bench.py per config).
#   bash scripts/gpu_r5m_configs.sh TAG "bench args" [TAG "bench args" ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${R5_OUT:-r5m}; mkdir -p $O
while [ $# -ge 2 ]; do
  tag=$1; args=$2; shift 2
  timeout -k 10 560 python -u bench.py $args > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  echo "$tag $(cut -c1-260 $O/$tag.json)"
done
