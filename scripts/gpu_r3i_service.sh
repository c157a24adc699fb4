#!/bin/bash
# Round 3: service paths against the engine on the same box - headline bench (engine alone),
# then gRPC clients -> llm.LLMService (engine in a pool worker) and clients -> Raft leader ->
# LLM, closed loop with 1024 clients in 8 processes and 6 batches of requests (steady-state
# rate over the 20-90 % window reported beside the whole-run rate).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/svc_engine.json 2> gpurun_out/svc_engine.err || { tail -5 gpurun_out/svc_engine.err; exit 1; }
cut -c1-300 gpurun_out/svc_engine.json
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 500 python scripts/service_bench.py --model llama-3-8b "$@" > gpurun_out/service_$tag.json 2> gpurun_out/service_$tag.err
  local rc=$?; tail -2 gpurun_out/service_$tag.err; python -c "
import json; d=json.load(open('gpurun_out/service_$tag.json'))
print('$tag', {k: d.get(k) for k in ('requests','errors','seconds','requests_per_s','gen_tokens_per_s','steady_requests_per_s','steady_gen_tokens_per_s','p50_latency_ms','p99_latency_ms')})"; return $rc
}
run direct_pool --backend pool --client-procs 8 --mode direct --requests 6144 --concurrency 1024 --max-batch 1024 || exit 1
run raft_pool --backend pool --client-procs 8 --mode raft --requests 6144 --concurrency 1024 --max-batch 1024 || exit 1
