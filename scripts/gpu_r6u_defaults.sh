#!/bin/bash
# Round 6: per-model prefill chunk defaults (Mixtral 32k with 32k-token MoE calls, 70B 36k) -
# MoE tests at the new chunk, then the Mixtral and 70B rows with no environment overrides.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6u; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "moe" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
M="--model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1"
L="--model llama-3-70b --workload ask --batch 256 --steps 2 --warmup 1"
bash scripts/gpu_r6h_configs.sh r6u mix_1024a "$M" mix_1024b "$M" \
  mix_256 "--model mixtral-8x7b --workload suggest --batch 256 --steps 3 --warmup 1" \
  l70_256a "$L" l70_256b "$L" l70_224 "--model llama-3-70b --workload ask --batch 224 --steps 2 --warmup 1" || exit 1
