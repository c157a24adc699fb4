#!/bin/bash
# Round 6: the remaining BASELINE rows on the final tree - summarize, Gemma-2B 1024, Llama-3-8B
# 1536, the co-located groups, the service paths via the Raft leader and saturated (1,280
# clients) against the same box's engine.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6s; mkdir -p $O
( while sleep 50; do date +%s >> $O/heartbeat; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
bash scripts/gpu_r6h_configs.sh r6s engine "--steps 6 --warmup 2" \
  sum_512 "--workload summarize --batch 512 --steps 3 --warmup 1" \
  sum_1024 "--workload summarize --batch 1024 --steps 3 --warmup 1" \
  gemma_1024 "--model gemma-2b --batch 1024 --steps 4 --warmup 1" \
  l8_1536 "--batch 1536 --steps 3 --warmup 1" || exit 1
timeout -k 10 500 python -u scripts/colocate_bench.py --smart-mem 0.3 --summary-mem 0.6 \
  --seconds 60 > $O/colocate.json 2> $O/colocate.err || { tail -30 $O/colocate.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/colocate.json'));print('colocate', {k: (v['tok_s'], v['p50_s'], v['p99_s']) for k, v in d['features'].items()})"
s() {  # tag, args
  local tag=$1; shift
  timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b "$@" > $O/svc_$tag.json 2> $O/svc_$tag.err || { echo "svc $tag failed"; tail -5 $O/svc_$tag.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/svc_$tag.json'));e=json.load(open('$O/engine.json'))['value'];print('svc $tag', d['gen_tokens_per_s'], round(100*d['gen_tokens_per_s']/e,1), '%', 'p50', d['p50_latency_ms'], 'p99', d['p99_latency_ms'], 'errors', d['errors'])"
}
s raft --backend pool --client-procs 8 --mode raft --requests 20480 --concurrency 1024 --max-batch 1024 &&
s sat1280 --backend pool --client-procs 8 --mode direct --requests 20480 --concurrency 1280 --max-batch 1024
