#!/bin/bash
# Round 4: the fused MoE grouped GEMM with non-temporal expert-weight loads (variants 3 / 4):
# fp32 tests, the Mixtral layer micro-benchmark, then the Mixtral suggestions wave at batch 1024
# with variant 4 vs the default pick.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4ah
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "moe" > gpurun_out/r4ah/tests.log 2>&1 || { tail -30 gpurun_out/r4ah/tests.log; exit 1; }
tail -1 gpurun_out/r4ah/tests.log
timeout -k 10 300 python -u scripts/moe_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4ah/moe_bench.log || exit 1
for v in 4 -1; do
  DRTC_MOE_VARIANT=$v timeout -k 10 500 python -u bench.py --model mixtral-8x7b --workload suggest --batch 1024 --steps 2 --warmup 1 \
    > gpurun_out/r4ah/mix_v$v.json 2> gpurun_out/r4ah/mix_v$v.err || { tail -5 gpurun_out/r4ah/mix_v$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4ah/mix_v$v.json')); print($v, d['value'], d['p50_latency_ms'])"
done
