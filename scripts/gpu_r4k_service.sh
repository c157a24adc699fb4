#!/bin/bash
# Round 4: closed-loop service path with burst gathering in the engine loop
# (DRTC_BURST_GAP_MS) against without, same box; engine headline for the ratio.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4k
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r4k/engine.json 2> gpurun_out/r4k/engine.err || { tail -5 gpurun_out/r4k/engine.err; exit 1; }
cut -c1-200 gpurun_out/r4k/engine.json
svc() {  # tag, gap_ms, args
  local tag=$1 gap=$2; shift 2
  DRTC_BURST_GAP_MS=$gap timeout -k 10 500 python scripts/service_bench.py --model llama-3-8b "$@" > gpurun_out/r4k/service_$tag.json 2> gpurun_out/r4k/service_$tag.err
  local rc=$?; tail -2 gpurun_out/r4k/service_$tag.err; python -c "
import json; d=json.load(open('gpurun_out/r4k/service_$tag.json'))
print('$tag', {k: d.get(k) for k in ('requests','errors','seconds','gen_tokens_per_s','p50_latency_ms','p99_latency_ms')}, d.get('replica_delta'))"; return $rc
}
A="--backend pool --client-procs 8 --requests 10240 --concurrency 1024 --max-batch 1024"
svc direct_g0 0 $A --mode direct && \
svc direct_g3 3 $A --mode direct && \
svc direct_g10 10 $A --mode direct && \
svc raft_g3 3 $A --mode raft
