#!/bin/bash
# Round 5: which combination of GPU test files leaves the pytest process aborting at exit
# ("terminate called without an active exception", r5ac): file groups in one pytest process each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5ad; mkdir -p $O
T=tests
run() {
  local tag=$1; shift
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/$tag.log 2>&1
  rc=$?
  echo "$tag rc=$rc $(grep -E 'passed|failed' $O/$tag.log | tail -1) abort=$(grep -c 'terminate called' $O/$tag.log)"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
  return 0
}
run A $T/test_custom_allreduce_gpu.py $T/test_expert_parallel_gpu.py $T/test_gemm_gpu.py
run B $T/test_kernels_gpu.py $T/test_model_gpu.py $T/test_model_real_shapes_gpu.py $T/test_service_gpu.py
run C $T/test_gemm_gpu.py $T/test_kernels_gpu.py
run D $T/test_kernels_gpu.py $T/test_service_gpu.py
run E $T/test_model_gpu.py $T/test_model_real_shapes_gpu.py $T/test_service_gpu.py
exit 0
