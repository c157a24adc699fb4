#!/bin/bash
# Round 3: Llama-3-70B ask-AI on one GPU between batch 192 and 256 (the 10 s deadline knee).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3y
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
run() { local tag=$1; shift; timeout -k 10 500 python -u bench.py "$@" > gpurun_out/r3y/$tag.json 2> gpurun_out/r3y/$tag.err || { tail -5 gpurun_out/r3y/$tag.err; return 1; }; python -c "import json;d=json.load(open('gpurun_out/r3y/$tag.json'));print('$tag', d['value'], d.get('p50_latency_ms'), d.get('p99_latency_ms'))"; }
run ask70b_224 --model llama-3-70b --workload ask --batch 224 --steps 2 --warmup 1 && \
run ask70b_208 --model llama-3-70b --workload ask --batch 208 --steps 2 --warmup 1
