#!/bin/bash
# Round 5: direct service path vs the engine on one box, sweeping the served engine's arrival
# gathering (DRTC_ADMIT_MIN_TOKENS / DRTC_ADMIT_MAX_MS; default 8192 / 100).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5x; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
echo "engine $(python3 -c "import json;print(json.load(open('$O/engine.json'))['value'])")"
for cfg in 8192:100 4096:50 2048:30 16384:150; do
  tok=${cfg%:*}; ms=${cfg#*:}
  DRTC_ADMIT_MIN_TOKENS=$tok DRTC_ADMIT_MAX_MS=$ms timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b \
    --backend pool --client-procs 8 --mode direct --requests 20480 --concurrency 1024 --max-batch 1024 \
    > $O/svc_$tok.json 2> $O/svc_$tok.err || { tail -5 $O/svc_$tok.err; exit 1; }
  echo "svc $cfg $(python3 -c "import json;d=json.load(open('$O/svc_$tok.json'));print(d['gen_tokens_per_s'],d['steady_gen_tokens_per_s'],d['p50_latency_ms'],d['replica_delta'])")"
done
