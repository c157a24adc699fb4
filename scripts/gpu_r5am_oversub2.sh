#!/bin/bash
# Round 5: two consecutive direct-service runs at 1,280 closed-loop clients over the 1,024-slot
# engine (the error kinds reported), against the headline engine run on the same box.
# (r5an: the same after the servers' pending-call queue fix.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${R5_OUT:-r5am}; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/engine.json'));print('engine', d['value'])"
for r in 1 2; do
  timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b --backend pool --client-procs 8 --mode direct \
    --requests 20480 --concurrency 1280 --max-batch 1024 > $O/svc_$r.json 2> $O/svc_$r.err || { tail -5 $O/svc_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/svc_$r.json'));e=json.load(open('$O/engine.json'))['value'];print('svc run $r', d['gen_tokens_per_s'], round(100*d['gen_tokens_per_s']/e,1), '%', 'p50', d['p50_latency_ms'], 'p99', d['p99_latency_ms'], 'errors', d['errors'], d['error_kinds'])"
done
