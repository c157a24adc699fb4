#!/bin/bash
# Round 4: re-tune every decode projection with the weight-prefetch forms in the candidate
# set, merge on the box, 70B ask-AI at 256 / 224, the headline, and lm_head on gemm_w4 v63.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4u
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u scripts/tune_xd.py --configs llama-3-8b:1,llama-3-70b:1,llama-3-70b:8,gemma-2b:1 \
  --out gpurun_out/r4u/xd_tuned.json > gpurun_out/r4u/tune.log 2>&1 || { tail -20 gpurun_out/r4u/tune.log; exit 1; }
tail -1 gpurun_out/r4u/tune.log
python scripts/tune_gemms.py --merge gpurun_out/r4u/xd_tuned.json || exit 1
timeout -k 10 150 python -u scripts/w4_probe.py --shape 1024,128256,4096 --arms lib,v63,v31 --iters 10 --rounds 5 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4u/lm_head.log
for b in 256 224; do
  timeout -k 10 600 python -u bench.py --model llama-3-70b --workload ask --batch $b --steps 3 --warmup 1 \
    > gpurun_out/r4u/b70_$b.json 2> gpurun_out/r4u/b70_$b.err || { tail -5 gpurun_out/r4u/b70_$b.err; exit 1; }
  cut -c1-300 gpurun_out/r4u/b70_$b.json
done
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4u/bench.json 2> gpurun_out/r4u/bench.err || exit 1
cut -c1-120 gpurun_out/r4u/bench.json
