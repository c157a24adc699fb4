#!/bin/bash
# Round 3, last tree: the deadline-bound secondary configs - Llama-3-70B ask-AI on one GPU at
# batch 192 / 256 (10 s node->LLM deadline) and Mixtral suggestions at batch 1024.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3y
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
run() { local tag=$1; shift; timeout -k 10 500 python -u bench.py "$@" > gpurun_out/r3y/$tag.json 2> gpurun_out/r3y/$tag.err || { tail -5 gpurun_out/r3y/$tag.err; return 1; }; python -c "import json;d=json.load(open('gpurun_out/r3y/$tag.json'));print('$tag', d['value'], d.get('p50_latency_ms'), d.get('p99_latency_ms'))"; }
run ask70b_256 --model llama-3-70b --workload ask --batch 256 --steps 1 --warmup 1 && \
run ask70b_192 --model llama-3-70b --workload ask --batch 192 --steps 1 --warmup 1 && \
run mixtral_1024 --model mixtral-8x7b --workload suggest --batch 1024 --steps 1 --warmup 1
