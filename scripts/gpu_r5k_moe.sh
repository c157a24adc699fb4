#!/bin/bash
# Round 5: MoE on gemm_xd's grouped mode (variant 3): fp32 tests, then scripts/moe_bench.py on
# Mixtral shapes (every variant and explicit xd forms against per-expert hipBLASLt).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5k; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "moe" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u scripts/moe_bench.py > $O/moe_bench.log 2>&1 || { tail -20 $O/moe_bench.log; exit 1; }
grep -v amdgpu.ids $O/moe_bench.log
