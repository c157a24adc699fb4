#!/bin/bash
# Round 4: TP=8 rehearsal (8 gloo ranks sharing ONE GPU) at decode batch 128, where the
# Llama-3-70B TP8 shard shapes take the tuned gemm_xd forms; checks that the sharded
# engines stay in lockstep and finish every request (throughput meaningless here).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out/r4x
export HSA_ENABLE_IPC_MODE_LEGACY=0 DRTC_DIST_BACKEND=gloo
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29631 bench.py --gpus 8 --tp 8 --no-graphs --steps 1 --warmup 0 --kv-fraction 0.02 \
  --model llama-3-70b --workload ask --batch 128 --max-new-tokens 8 --custom-allreduce \
  > gpurun_out/r4x/tp8_70b_b128.json 2> gpurun_out/r4x/tp8_70b_b128.err
rc=$?; [ $rc -eq 0 ] || { tail -30 gpurun_out/r4x/tp8_70b_b128.err; exit $rc; }
cut -c1-600 gpurun_out/r4x/tp8_70b_b128.json
