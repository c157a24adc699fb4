#!/bin/bash
# Round 3: service paths with the native tokenizer (csrc/runtime/tokenizer.cpp, GIL released
# in the engine worker) against the Python tokenizer, same box; engine headline for the ratio.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3u
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3u/engine.json 2> gpurun_out/r3u/engine.err || { tail -5 gpurun_out/r3u/engine.err; exit 1; }
cut -c1-200 gpurun_out/r3u/engine.json
svc() {  # tag, env, args
  local tag=$1 envs=$2; shift 2
  env $envs timeout -k 10 500 python scripts/service_bench.py --model llama-3-8b "$@" > gpurun_out/r3u/service_$tag.json 2> gpurun_out/r3u/service_$tag.err
  local rc=$?; tail -2 gpurun_out/r3u/service_$tag.err; python -c "
import json; d=json.load(open('gpurun_out/r3u/service_$tag.json'))
print('$tag', {k: d.get(k) for k in ('requests','errors','seconds','gen_tokens_per_s','steady_gen_tokens_per_s','p50_latency_ms','p99_latency_ms')}, d.get('replica_delta'))"; return $rc
}
A="--backend pool --client-procs 8 --requests 6144 --concurrency 1024 --max-batch 1024"
svc direct_native DRTC_NATIVE_TOKENIZER=1 $A --mode direct && \
svc direct_py DRTC_NATIVE_TOKENIZER=0 $A --mode direct && \
svc direct_native_aio DRTC_NATIVE_TOKENIZER=1 $A --mode direct --frontend aio && \
svc raft_native DRTC_NATIVE_TOKENIZER=1 $A --mode raft
