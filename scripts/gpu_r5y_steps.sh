#!/bin/bash
# Round 5: host wall time per engine step kind (stats[<kind>_us]) in the headline bench and in
# a direct-service run on the same box: where the served engine's closed loop loses time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5y; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/engine.json'));print('engine', d['value'], d['engine_stats'])"
timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b --backend pool --client-procs 8 --mode direct \
  --requests 20480 --concurrency 1024 --max-batch 1024 > $O/svc.json 2> $O/svc.err || { tail -5 $O/svc.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/svc.json'));print('svc', d['gen_tokens_per_s'], d['seconds'], d['replica_delta'])"
