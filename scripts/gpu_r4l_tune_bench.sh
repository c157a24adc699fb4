#!/bin/bash
# Round 4: tune gemm_xd per model decode shape, merge into the table on the box, then the
# headline A/B on one box: xd + variant 31 (default), without xd, and variant 15.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4l
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py -k "xd or norm_glu" > gpurun_out/r4l/tests_xd.log 2>&1 || { tail -30 gpurun_out/r4l/tests_xd.log; exit 1; }
tail -1 gpurun_out/r4l/tests_xd.log
timeout -k 10 900 python -u scripts/tune_xd.py --configs llama-3-8b:1,gemma-2b:1,llama-3-70b:1,llama-3-70b:8 \
  --out gpurun_out/r4l/xd_tuned.json > gpurun_out/r4l/tune.log 2>&1 || { tail -20 gpurun_out/r4l/tune.log; exit 1; }
grep -c xd_form gpurun_out/r4l/tune.log; tail -1 gpurun_out/r4l/tune.log
python scripts/tune_gemms.py --merge gpurun_out/r4l/xd_tuned.json || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py -k "router or off_bucket or persistent" > gpurun_out/r4l/tests.log 2>&1 || { tail -30 gpurun_out/r4l/tests.log; exit 1; }
tail -1 gpurun_out/r4l/tests.log
b() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4l/bench_$tag.json 2> gpurun_out/r4l/bench_$tag.err || { tail -5 gpurun_out/r4l/bench_$tag.err; return 1; }
  echo $tag $(cut -c1-160 gpurun_out/r4l/bench_$tag.json)
}
b xd DRTC_XD_GEMM=1 && b noxd DRTC_XD_GEMM=0 && b xd_v15 DRTC_W4_VARIANT=15 && b xd2 DRTC_XD_GEMM=1
