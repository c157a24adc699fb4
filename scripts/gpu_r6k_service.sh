#!/bin/bash
# Round 6: the direct service path with ONE closed-loop client per engine
# slot (1,024) against the headline engine on the same box - front-end / backend / admission
# variants, one run each:  R6K_ARMS="tag:frontend:backend:ENV=VAL,..." (space-separated).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${R6K_OUT:-r6k}; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/engine.json'));print('engine', d['value'])"
for arm in ${R6K_ARMS:-threads_pool:threads:pool: aio_pool:aio:pool: threads_engine:threads:engine:}; do
  IFS=: read tag fe be envs <<< "$arm"
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b --backend $be --frontend $fe \
    --client-procs 8 --mode direct --requests 20480 --concurrency 1024 --max-batch 1024 > $O/svc_$tag.json 2> $O/svc_$tag.err || { tail -5 $O/svc_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/svc_$tag.json'));e=json.load(open('$O/engine.json'))['value'];print('svc $tag', d['gen_tokens_per_s'], round(100*d['gen_tokens_per_s']/e,1), '%', 'steady', d['steady_gen_tokens_per_s'], 'p50', d['p50_latency_ms'], 'errors', d['errors'])"
done
