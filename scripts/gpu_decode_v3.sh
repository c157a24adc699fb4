#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_kernels_gpu.py -k paged_decode > gpurun_out/decode_v3_tests.log 2>&1
rc=$?; tail -5 gpurun_out/decode_v3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/decode_attn_bench.py 1,2,3 > gpurun_out/decode_v3_bench.log 2>&1
rc=$?; cat gpurun_out/decode_v3_bench.log; exit $rc
