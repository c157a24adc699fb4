#!/bin/bash
# Round 5: the remaining Llama-3-8B BASELINE rows (batch 256 / 512 / 1536, small batches) and
# both service paths (closed loop, 1024 clients in 8 processes, engine in a worker process).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5o; mkdir -p $O
b() {  # tag, args
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  echo "$tag $(python3 -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['p50_latency_ms'])")"
}
s() {  # tag, args
  local tag=$1; shift
  timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b "$@" > $O/svc_$tag.json 2> $O/svc_$tag.err || { echo "svc $tag failed"; tail -5 $O/svc_$tag.err; return 1; }
  echo "svc $tag $(python3 -c "import json;d=json.load(open('$O/svc_$tag.json'));print(d['gen_tokens_per_s'],d['p50_latency_ms'],d['p99_latency_ms'])")"
}
b engine1024 --steps 6 --warmup 2 &&
s direct --backend pool --client-procs 8 --mode direct --requests 10240 --concurrency 1024 --max-batch 1024 &&
s raft --backend pool --client-procs 8 --mode raft --requests 10240 --concurrency 1024 --max-batch 1024 &&
b b512 --batch 512 --steps 4 --warmup 1 &&
b b256 --batch 256 --steps 4 --warmup 1 &&
b b1536 --batch 1536 --steps 3 --warmup 1 &&
b b1 --batch 1 --steps 3 --warmup 1 &&
b b16 --batch 16 --steps 3 --warmup 1
