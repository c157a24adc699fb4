#!/bin/bash
# Round 5: direct service path vs the engine loop on ONE box: bench.py, then two consecutive
# closed-loop runs of 20 waves (20480 requests, 1024 clients in 8 processes); then the gemm_w4
# per-tile overhead probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
echo "engine $(python3 -c "import json;d=json.load(open('$O/engine.json'));print(d['value'])")"
for r in 1 2; do
  timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b --backend pool --client-procs 8 --mode direct \
    --requests 20480 --concurrency 1024 --max-batch 1024 > $O/svc_direct_$r.json 2> $O/svc_direct_$r.err || { tail -5 $O/svc_direct_$r.err; exit 1; }
  echo "svc direct $r $(python3 -c "import json;d=json.load(open('$O/svc_direct_$r.json'));print(d['gen_tokens_per_s'],d['steady_gen_tokens_per_s'],d['p50_latency_ms'],d['replica_delta'])")"
done
bash scripts/gpu_r5q_seam.sh
