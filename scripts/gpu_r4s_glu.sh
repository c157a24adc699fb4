#!/bin/bash
# Round 4: tune the gated gemm_xd forms for gate_up at every decode bucket (against gemm_w4's
# fused GLU from 640 rows, the library + act_glu below), merge on the box, re-run the GEMM and
# model tests, then the headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4s
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u scripts/tune_xd.py --gemms gate_up --configs llama-3-8b:1,gemma-2b:1,llama-3-70b:1,llama-3-70b:8 \
  --out gpurun_out/r4s/xd_glu_tuned.json > gpurun_out/r4s/tune.log 2>&1 || { tail -20 gpurun_out/r4s/tune.log; exit 1; }
tail -1 gpurun_out/r4s/tune.log
python scripts/tune_gemms.py --merge gpurun_out/r4s/xd_glu_tuned.json || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_model_gpu.py > gpurun_out/r4s/tests.log 2>&1 || { tail -30 gpurun_out/r4s/tests.log; exit 1; }
tail -1 gpurun_out/r4s/tests.log
for t in a b; do
  timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4s/bench_$t.json 2> gpurun_out/r4s/bench_$t.err || { tail -5 gpurun_out/r4s/bench_$t.err; exit 1; }
  cut -c1-120 gpurun_out/r4s/bench_$t.json
done
