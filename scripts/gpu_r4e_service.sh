#!/bin/bash
# Round 4: service paths with K gRPC front-end processes on one port (llm/frontends.py)
# against the single front-end, same box; engine headline for the ratio.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4e
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r4e/engine.json 2> gpurun_out/r4e/engine.err || { tail -5 gpurun_out/r4e/engine.err; exit 1; }
cut -c1-200 gpurun_out/r4e/engine.json
svc() {  # tag, args
  local tag=$1; shift
  timeout -k 10 500 python scripts/service_bench.py --model llama-3-8b "$@" > gpurun_out/r4e/service_$tag.json 2> gpurun_out/r4e/service_$tag.err
  local rc=$?; tail -2 gpurun_out/r4e/service_$tag.err; python -c "
import json; d=json.load(open('gpurun_out/r4e/service_$tag.json'))
print('$tag', {k: d.get(k) for k in ('requests','errors','seconds','gen_tokens_per_s','steady_gen_tokens_per_s','p50_latency_ms','p99_latency_ms')}, d.get('replica_delta'))"; return $rc
}
A="--backend pool --client-procs 8 --requests 6144 --concurrency 1024 --max-batch 1024"
svc direct_fe4 $A --mode direct --frontends 4 && \
svc direct_fe1 $A --mode direct && \
svc raft_fe4 $A --mode raft --frontends 4 && \
svc direct_fe8 $A --mode direct --frontends 8
