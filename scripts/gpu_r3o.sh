#!/bin/bash
# Round 3: model / GEMM tests after the folded-norm opt-in change, then the service paths with
# tokenization + detokenization moved into the engine worker process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_gemm_gpu.py -q --timeout 200 --timeout-method thread -k "residual or rinv or rs_linear or folded or partials" > gpurun_out/t_r3o.log 2>&1
rc=$?; tail -3 gpurun_out/t_r3o.log; [ $rc -le 1 ] || exit $rc
bash scripts/gpu_r3i_service.sh
