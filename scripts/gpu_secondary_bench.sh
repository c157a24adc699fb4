#!/bin/bash
# GPU model tests, then timed bench.py runs of the secondary BASELINE configs.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_model_gpu.py tests/test_model_real_shapes_gpu.py > gpurun_out/sec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sec_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, bench args...
  local tag=$1; shift
  DRTC_TIME_DECODE=1 timeout -k 10 400 python bench.py "$@" > gpurun_out/sec_$tag.json 2> gpurun_out/sec_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/sec_$tag.err; exit 1; }
  echo "$tag $(cut -c1-200 gpurun_out/sec_$tag.json)"; grep "decode graph" gpurun_out/sec_$tag.err
}
run gemma --model gemma-2b && \
run mixtral --model mixtral-8x7b --workload suggest --batch 256 && \
run ask70b --model llama-3-70b --workload ask --batch 256 --steps 1
