#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_kernels_gpu.py -k prefill > gpurun_out/pp_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" gpurun_out/pp_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/prefill_attn_bench.py > gpurun_out/pp_bench.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/pp_bench.log; exit $rc
