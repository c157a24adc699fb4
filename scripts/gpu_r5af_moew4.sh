#!/bin/bash
# Round 5: MoE variant 4 (token rows gathered into expert order, expert GEMMs on gemm_w4's
# grouped mode): fp32 tests, moe_bench at Mixtral shapes from decode to prefill T, then the
# Mixtral suggestions wave at batch 1024.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5af; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gemm_gpu.py -k "moe or w4 or mfma_gemm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python -u scripts/moe_bench.py 14336 512,1024,2048,4096,8192,16384 > $O/moe_bench.log 2>&1 || { tail -20 $O/moe_bench.log; exit 1; }
grep "^T=" $O/moe_bench.log | cut -c1-140
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1 \
  > $O/mixtral1024.json 2> $O/mixtral1024.err || { tail -5 $O/mixtral1024.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/mixtral1024.json'));print('mixtral', d['value'], d.get('p50_latency_ms'))"
