#!/bin/bash
# Round 5: gemm_xd 1x8 (128 x 256, 3-slot ring) form - fp32 tests, MoE forms on Mixtral shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_gemm_gpu.py -k "moe or xd_gemm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u scripts/moe_bench.py 14336 256,512,1024,2048 > $O/moe_bench.log 2>&1 || { tail -20 $O/moe_bench.log; exit 1; }
grep -v amdgpu.ids $O/moe_bench.log | cut -c1-400
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
$P --shape 1024,28672,4096 --epi silu --rotate 3 --arms v63,x281,x181,x1181 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | cut -c1-200
