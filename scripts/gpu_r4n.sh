#!/bin/bash
# Round 4: re-run the kernel tests that injected old-width table entries, prefill PMC
# comparison (gemm_w4 vs hipBLASLt), then the service burst-gathering A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4n
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "skinny_norm_gemm or skinny_glu_gemm or tuned_linear" > gpurun_out/r4n/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4n/tests.log; [ $rc -le 1 ] || exit $rc
bash scripts/gpu_r4j_pmc.sh || exit 1
bash scripts/gpu_r4k_service.sh
