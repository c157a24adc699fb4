#!/bin/bash
# Round 4: Mixtral decode MoE grouped-GEMM variant at T = 1024: the micro-benchmark twice, then
# the suggestions wave at batch 1024 with variant 0 vs the default pick (2), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4ak
timeout -k 10 300 python -u scripts/moe_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4ak/moe_bench.log || exit 1
for v in 0 -1 0 -1; do
  DRTC_MOE_VARIANT=$v timeout -k 10 500 python -u bench.py --model mixtral-8x7b --workload suggest --batch 1024 --steps 2 --warmup 1 \
    > gpurun_out/r4ak/mix_v$v.json 2> gpurun_out/r4ak/mix_v$v.err || { tail -5 gpurun_out/r4ak/mix_v$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4ak/mix_v$v.json')); print($v, d['value'], d['p50_latency_ms'])" | tee -a gpurun_out/r4ak/mix.log
done
