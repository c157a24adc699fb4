#!/bin/bash
# Round 3: the EP default path (capacity-factor all-to-all in prefill and decode) - TP8/EP8
# rehearsal with 8 gloo ranks on one GPU (correctness only), then Mixtral on one GPU (no EP,
# fused MoE without host syncs) timed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u bench.py --model mixtral-8x7b --workload suggest --batch 1024 --steps 2 --warmup 1 > gpurun_out/mixtral_b1024.json 2> gpurun_out/mixtral_b1024.err || { tail -5 gpurun_out/mixtral_b1024.err; exit 1; }
cut -c1-330 gpurun_out/mixtral_b1024.json; echo
bash scripts/gpu_tp8_rehearsal.sh
