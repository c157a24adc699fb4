#!/bin/bash
# Paged decode attention variants 1/2/3 at the Gemma-2B / Mixtral / Llama-3-70B bench
# geometries (after the decode-kernel tests pass).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_kernels_gpu.py -k paged_decode > gpurun_out/decode_geoms_tests.log 2>&1
rc=$?; tail -3 gpurun_out/decode_geoms_tests.log; [ $rc -eq 0 ] || exit $rc
for g in gemma mixtral llama70b; do
  timeout -k 10 300 python -u scripts/decode_attn_bench.py 1,2,3 $g >> gpurun_out/decode_geoms_bench.log 2>&1 || exit $?
done
cat gpurun_out/decode_geoms_bench.log
