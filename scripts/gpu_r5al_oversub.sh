#!/bin/bash
# Round 5: direct service throughput at the engine's batch (1,024 slots) with the closed loop
# exactly filling the slots vs oversubscribed (requests waiting in the engine's queue while
# finished ones travel back), same box, against the headline engine run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5al; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/engine.json'));print('engine', d['value'])"
for c in 1024 1280 1536; do
  timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b --backend pool --client-procs 8 --mode direct \
    --requests 20480 --concurrency $c --max-batch 1024 > $O/svc_$c.json 2> $O/svc_$c.err || { tail -5 $O/svc_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/svc_$c.json'));e=json.load(open('$O/engine.json'))['value'];print('svc c=$c', d['gen_tokens_per_s'], round(100*d['gen_tokens_per_s']/e,1), '%', 'p50', d.get('p50_ms'), 'p99', d.get('p99_ms'))"
done
