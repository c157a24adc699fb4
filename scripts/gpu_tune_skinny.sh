#!/bin/bash
# Skinny-vs-library pick for every small-batch decode GEMM of the served models.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "llama-3-8b 1" "llama-3-70b 1" "llama-3-70b 8" "gemma-2b 1" "mixtral-8x7b 1" "llama-3-8b 2" "llama-3-8b 4" "llama-3-8b 8"; do
  set -- $spec
  timeout -k 10 300 python -u scripts/tune_skinny.py --model $1 --tp $2 --ms 1,2,4,8,16 --out gpurun_out/skinny_tuned.json >> gpurun_out/tune_skinny.log 2>&1 || exit $?
done
