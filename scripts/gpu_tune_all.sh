#!/bin/bash
# Tune every decode projection GEMM (all hipGraph buckets) of the served models.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "llama-3-8b 1" "llama-3-70b 1" "llama-3-70b 8" "gemma-2b 1" "mixtral-8x7b 1" "llama-3-8b 2" "llama-3-8b 4" "llama-3-8b 8"; do
  set -- $spec
  timeout -k 10 400 python -u scripts/tune_gemms.py --model $1 --tp $2 --out gpurun_out/tuned_$1_tp$2.json >> gpurun_out/tune_all.log 2>&1 || exit $?
done
