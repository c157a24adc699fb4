#!/bin/bash
# Round 4: GEMM / model GPU tests + smoke on the pruned GEMM set, the seam experiment, and
# the Gemma-2B batch-2048 decode GEMM tuning (its server default batch, above the 1024 buckets).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r4d
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4d
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py "tests/test_kernels_gpu.py::test_paged_decode_fused_rope" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u scripts/tune_gemms.py --model gemma-2b --ms 1536,2048 --out $O/gemma2048.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -3 $O/tune.log
timeout -k 10 600 bash scripts/gpu_r4b_seam.sh > $O/seam.log 2>&1 || { tail -20 $O/seam.log; exit 1; }
cat $O/seam.log
