#!/bin/bash
# Round 4: the 70B ask wave at batch 256 with prefill chunks of 16k (default), 24k and 36k tokens.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4ag
for c in 36864 24576 16384; do
  DRTC_PREFILL_CHUNK=$c timeout -k 10 600 python -u bench.py --model llama-3-70b --workload ask --batch 256 --steps 3 --warmup 1 \
    > gpurun_out/r4ag/b70_c$c.json 2> gpurun_out/r4ag/b70_c$c.err || { tail -5 gpurun_out/r4ag/b70_c$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4ag/b70_c$c.json')); print($c, d['value'], d['p50_latency_ms'], d['p50_ttft_ms'])"
done
