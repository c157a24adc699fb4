#!/bin/bash
# Serving under load on one MI355X: engine-level open loop (bench.py
# --arrival-rate) at two rates, then the gRPC service paths (closed loop with
# 1024 clients in 8 processes, direct and through the Raft leader; open loop
# through the Raft leader).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ol() {  # rate, extra args
  local rate=$1; shift
  timeout -k 10 300 python -u bench.py --warmup 1 --arrival-rate "$rate" --requests $((rate * 15)) "$@" \
    > gpurun_out/ss_ol_$rate.json 2> gpurun_out/ss_ol_$rate.err || { echo "ol $rate failed"; tail -5 gpurun_out/ss_ol_$rate.err; return 1; }
  cut -c1-700 gpurun_out/ss_ol_$rate.json
}
svc() {  # tag, args
  local tag=$1; shift
  timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b "$@" > gpurun_out/ss_svc_$tag.json 2> gpurun_out/ss_svc_$tag.err \
    || { echo "svc $tag failed"; tail -5 gpurun_out/ss_svc_$tag.err; return 1; }
  cut -c1-520 gpurun_out/ss_svc_$tag.json; echo
}
ol 300 && ol 400 \
  && svc direct_pool --backend pool --client-procs 8 --mode direct --requests 3072 --concurrency 1024 --max-batch 1024 \
  && svc raft_pool --backend pool --client-procs 8 --mode raft --requests 3072 --concurrency 1024 --max-batch 1024 \
  && svc raft_pool_open300 --backend pool --mode raft --requests 4500 --arrival-rate 300 --max-batch 1024
