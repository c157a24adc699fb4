#!/bin/bash
# Round 3: where the closed-loop service loses against the closed-wave engine - replica idle
# time per run (engine counters), at 1024 clients (= engine batch) and at 1536 clients.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 500 python scripts/service_bench.py --model llama-3-8b "$@" > gpurun_out/service_$tag.json 2> gpurun_out/service_$tag.err
  local rc=$?; tail -2 gpurun_out/service_$tag.err; python -c "
import json; d=json.load(open('gpurun_out/service_$tag.json'))
print('$tag', {k: d.get(k) for k in ('requests','seconds','requests_per_s','gen_tokens_per_s','p50_latency_ms','p99_latency_ms','replica_delta')})"; return $rc
}
run direct_pool_c1024 --backend pool --client-procs 8 --mode direct --requests 6144 --concurrency 1024 --max-batch 1024 || exit 1
run direct_pool_c1536 --backend pool --client-procs 8 --mode direct --requests 9216 --concurrency 1536 --max-batch 1024 || exit 1
