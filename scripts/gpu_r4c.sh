#!/bin/bash
# Round 4: the pruned GEMM set + router on MI355X (GEMM / model GPU tests, smoke), then the
# prefill seam experiment (persistent gemm_w4 with / without the per-XCD K rotation).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r4c
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4c
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 bash scripts/gpu_r4b_seam.sh > $O/seam.log 2>&1 || { tail -20 $O/seam.log; exit 1; }
cat $O/seam.log
