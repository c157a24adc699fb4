#!/bin/bash
# Round 5: fused MoE reads the router GEMM's [E, T] output in place (no transpose copy per
# layer): MoE / router / EP tests, then the Mixtral suggestions wave at batch 1024 twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5at; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_expert_parallel_gpu.py -k "router or moe or ep_" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 600 python -u bench.py --model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1 \
    > $O/mixtral1024_$r.json 2> $O/mixtral1024_$r.err || { tail -5 $O/mixtral1024_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/mixtral1024_$r.json'));print('mixtral view', d['value'], d.get('p50_latency_ms'))"
done
