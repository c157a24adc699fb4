#!/bin/bash
# Multi-rank rehearsal on ONE GPU (the 8-GPU node is the driver's): two ranks
# share cuda:0 over the gloo backend (RCCL refuses two ranks per device).
#  * TP=2 Llama-3-8B: sharded weights, TP kernels, the IPC one-shot all-reduce
#    for decode-sized messages, gloo for prefill all-reduces / logits gather
#    (eager decode: gloo collectives cannot be graph-captured);
#  * DP=2 bench.py: the driver's scaling launch (torchrun, max-over-ranks timing).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DRTC_DIST_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 400 $TR --master-port 29611 bench.py --gpus 2 --tp 2 --custom-allreduce --no-graphs \
  --batch 64 --steps 1 --warmup 1 --kv-fraction 0.3 > gpurun_out/rehearsal_tp2.json 2> gpurun_out/rehearsal_tp2.err \
  || { echo "tp2 failed"; tail -20 gpurun_out/rehearsal_tp2.err; exit 1; }
cut -c1-300 gpurun_out/rehearsal_tp2.json
timeout -k 10 400 $TR --master-port 29612 bench.py --gpus 2 --batch 256 --steps 1 --warmup 1 \
  --kv-fraction 0.3 > gpurun_out/rehearsal_dp2.json 2> gpurun_out/rehearsal_dp2.err \
  || { echo "dp2 failed"; tail -20 gpurun_out/rehearsal_dp2.err; exit 1; }
cut -c1-300 gpurun_out/rehearsal_dp2.json
