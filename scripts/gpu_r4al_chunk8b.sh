#!/bin/bash
# Round 4: headline with prefill chunks of 16k (default) / 24k / 32k tokens, interleaved on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4al
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in 32768 16384 24576 32768 16384; do
  DRTC_PREFILL_CHUNK=$c timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 > gpurun_out/r4al/b_$c.json 2> gpurun_out/r4al/b_$c.err || { tail -5 gpurun_out/r4al/b_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4al/b_$c.json')); print($c, d['value'], d['p50_latency_ms'], d['engine_stats'])" | tee -a gpurun_out/r4al/chunk.log
done
