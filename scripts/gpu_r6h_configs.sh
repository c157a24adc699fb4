#!/bin/bash
# Round 6: re-measure the BASELINE rows on the final tree (one timed bench.py per config).
#   bash scripts/gpu_r6h_configs.sh OUT TAG "bench args" [TAG "bench args" ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/$1; shift; mkdir -p $O
while [ $# -ge 2 ]; do
  tag=$1; args=$2; shift 2
  timeout -k 10 560 python -u bench.py $args > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'], d['p50_latency_ms'], d.get('p50_ttft_ms'))")"
done
