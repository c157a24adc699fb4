#!/bin/bash
# Round 6: MoE variant 4 as the default from 256 rows per expert, 16k-token MoE chunks - tests,
# the prefill layer (+ K-rotation A/B), moe_bench at decode sizes, Mixtral waves at 1024 / 256.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6l; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py -k "grouped or moe" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/moe_prefill_anatomy.py 16384 > $O/anat16k.log 2>&1 || { tail -20 $O/anat16k.log; exit 1; }
grep "^T=" $O/anat16k.log
timeout -k 10 400 python -u scripts/moe_bench.py 14336 256,512,1024 > $O/moe_bench.log 2>&1 || { tail -20 $O/moe_bench.log; exit 1; }
grep "^T=" $O/moe_bench.log | cut -c1-400
bash scripts/gpu_r6h_configs.sh r6l mix_1024a "--model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1" \
  mix_1024b "--model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1" \
  mix_256 "--model mixtral-8x7b --workload suggest --batch 256 --steps 3 --warmup 1" || exit 1
