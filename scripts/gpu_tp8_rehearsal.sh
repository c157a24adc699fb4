#!/bin/bash
# TP=8 rehearsal on ONE GPU (the 8-GPU node is the driver's): eight ranks share
# cuda:0 over the gloo backend (RCCL refuses two ranks per device), each holding
# its 1/8 shard, so the exact TP=8 code path of the two multi-GPU configs runs:
#  * Llama-3-70B ask-AI, TP=8: column/row-sharded projections (hq 8, hkv 1 per
#    rank), the IPC all-reduce with 8 peers for decode-sized messages, gloo for
#    prefill all-reduces and the logits gather;
#  * Mixtral 8x7B suggestions, TP=8 + EP=8: one expert per rank, the expert
#    all-to-all (parallel/expert_parallel.py) on the prefill path.
# Eight processes time-slice one GPU and gloo moves prefill activations through
# host memory, so the throughput printed here means nothing; the run checks that
# the sharded engines start, stay in lockstep and finish every request.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DRTC_DIST_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1"
run() {  # name, port, bench args...
  local name=$1 port=$2; shift 2
  timeout -k 10 540 $TR --master-port "$port" bench.py --gpus 8 --tp 8 --no-graphs \
    --steps 1 --warmup 0 --kv-fraction 0.02 "$@" \
    > "gpurun_out/rehearsal_$name.json" 2> "gpurun_out/rehearsal_$name.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -30 "gpurun_out/rehearsal_$name.err"; return $rc; fi
  cut -c1-400 "gpurun_out/rehearsal_$name.json"
}
run tp8_70b 29621 --model llama-3-70b --workload ask --batch 8 --max-new-tokens 24 --custom-allreduce \
  && run tp8_mixtral 29622 --model mixtral-8x7b --workload suggest --batch 8 --max-new-tokens 24 --custom-allreduce
