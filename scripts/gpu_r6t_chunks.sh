#!/bin/bash
# Round 6: prefill chunk size A/B on one box - Mixtral (32k-token prefill steps and MoE calls:
# 8k rows per expert) and Llama-3-70B (one ~35k-token prefill step per ask wave).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
M="--model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1"
L="--model llama-3-70b --workload ask --batch 256 --steps 2 --warmup 1"
bash scripts/gpu_r6h_configs.sh r6t mix_c16 "$M" || exit 1
DRTC_PREFILL_CHUNK=32768 DRTC_MOE_CHUNK=32768 bash scripts/gpu_r6h_configs.sh r6t mix_c32 "$M" || exit 1
bash scripts/gpu_r6h_configs.sh r6t mix_c16b "$M" || exit 1
DRTC_PREFILL_CHUNK=32768 DRTC_MOE_CHUNK=32768 bash scripts/gpu_r6h_configs.sh r6t mix_c32b "$M" || exit 1
bash scripts/gpu_r6h_configs.sh r6t l70_c16 "$L" || exit 1
DRTC_PREFILL_CHUNK=36864 bash scripts/gpu_r6h_configs.sh r6t l70_c36 "$L" || exit 1
