#!/bin/bash
# Round 6: Llama-3-8B batch 1536 with gemm_xd forms for its 1536-row decode o / down
# (DRTC_XD_BIG_M=0 = the previous library route), interleaved on one box; router GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6an; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
G="--batch 1536 --steps 3 --warmup 1"
for r in 1 2; do
  DRTC_XD_BIG_M=0 bash scripts/gpu_r6h_configs.sh r6an lib_$r "$G" || exit 1
  bash scripts/gpu_r6h_configs.sh r6an xd_$r "$G" || exit 1
done
