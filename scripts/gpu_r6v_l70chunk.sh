#!/bin/bash
# Round 6: Llama-3-70B prefill step A/B on one box, interleaved - 16k steps vs the model
# default (one 36k step per wave), at batch 224 (the server default) and 256.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
A="--model llama-3-70b --workload ask --steps 2 --warmup 1"
for r in 1 2; do
  DRTC_PREFILL_CHUNK=16384 bash scripts/gpu_r6h_configs.sh r6v b224_c16_$r "$A --batch 224" || exit 1
  bash scripts/gpu_r6h_configs.sh r6v b224_c36_$r "$A --batch 224" || exit 1
  DRTC_PREFILL_CHUNK=16384 bash scripts/gpu_r6h_configs.sh r6v b256_c16_$r "$A --batch 256" || exit 1
  bash scripts/gpu_r6h_configs.sh r6v b256_c36_$r "$A --batch 256" || exit 1
done
