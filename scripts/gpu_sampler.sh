#!/bin/bash
# Sampler numerics (GPU tests) then timing per mode at the headline shape.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_kernels_gpu.py -k sample > gpurun_out/sampler_tests.log 2>&1 \
  && tail -12 gpurun_out/sampler_tests.log \
  && timeout -k 10 200 python -u scripts/sampler_bench.py > gpurun_out/sampler_bench.log 2>&1 \
  && cat gpurun_out/sampler_bench.log
