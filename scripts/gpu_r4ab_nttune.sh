#!/bin/bash
# Round 4: re-tune gemm_xd at the decode buckets that fit one 256-row tile with the
# non-temporal forms among the candidates (Llama-3-70B TP1 / TP8, Llama-3-8B, Gemma-2B), merge,
# then the 70B ask-AI wave at batch 256 / 224 and the headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4ab
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u scripts/tune_xd.py --configs llama-3-70b:1,llama-3-70b:8,llama-3-8b:1,gemma-2b:1 \
  --ms 128,160,192,224,256 --out gpurun_out/r4ab/xd_tuned.json 2>&1 | grep -v amdgpu.ids > gpurun_out/r4ab/tune.log || exit 1
tail -1 gpurun_out/r4ab/tune.log
python scripts/tune_gemms.py --merge gpurun_out/r4ab/xd_tuned.json || exit 1
for b in 256 224; do
  timeout -k 10 600 python -u bench.py --model llama-3-70b --workload ask --batch $b --steps 3 --warmup 1 \
    > gpurun_out/r4ab/b70_$b.json 2> gpurun_out/r4ab/b70_$b.err || { tail -5 gpurun_out/r4ab/b70_$b.err; exit 1; }
  cut -c1-200 gpurun_out/r4ab/b70_$b.json
done
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r4ab/engine.json 2> gpurun_out/r4ab/engine.err || exit 1
cut -c1-160 gpurun_out/r4ab/engine.json
cp distributed-real-time-chat-and-collaboration-tool_amd/ops/tuned/gemm_gfx950.json gpurun_out/r4ab/
