#!/bin/bash
# Service-level load driver on Llama-3-8B: gRPC clients -> llm.LLMService
# directly, and through the Raft leader (raft.RaftNode/GetSmartReply).
# Clients run in 8 separate processes; "pool" keeps the engine in its own
# process (the server process only does gRPC, prompts, tokenization, parsing).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 600 python scripts/service_bench.py --model llama-3-8b "$@" > gpurun_out/service_$tag.json 2> gpurun_out/service_$tag.err
  local rc=$?; tail -2 gpurun_out/service_$tag.err; cut -c1-420 gpurun_out/service_$tag.json; echo; return $rc
}
run direct_inproc --mode direct --requests 2048 --concurrency 1024 --max-batch 1024 || exit 1
run direct_pool --backend pool --client-procs 8 --mode direct --requests 2048 --concurrency 1024 --max-batch 1024 || exit 1
run raft_pool --backend pool --client-procs 8 --mode raft --requests 2048 --concurrency 1024 --max-batch 1024 || exit 1
# open loop (Poisson) through the Raft leader: latency from the scheduled send
run raft_pool_open300 --backend pool --mode raft --requests 4500 --arrival-rate 300 --max-batch 1024 || exit 1
