#!/bin/bash
# Round 4: re-run the table-injecting kernel tests, lm_head on gemm_w4 v63 vs the library, and
# the direct service path twice more (run-to-run spread of the closed loop).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4v
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "skinny or tuned_linear" > gpurun_out/r4v/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4v/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 150 python -u scripts/w4_probe.py --shape 1024,128256,4096 --arms lib,v63,v31 --iters 10 --rounds 5 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4v/lm_head.log || exit 1
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r4v/engine.json 2> gpurun_out/r4v/engine.err || exit 1
cut -c1-120 gpurun_out/r4v/engine.json
for t in a b; do
  timeout -k 10 500 python scripts/service_bench.py --model llama-3-8b --backend pool --client-procs 8 \
    --requests 10240 --concurrency 1024 --max-batch 1024 --mode direct > gpurun_out/r4v/service_$t.json 2> gpurun_out/r4v/service_$t.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/r4v/service_$t.json'))
print('$t', {k: d.get(k) for k in ('requests','errors','seconds','gen_tokens_per_s','p50_latency_ms','p99_latency_ms')}, d.get('replica_delta'))"
done
