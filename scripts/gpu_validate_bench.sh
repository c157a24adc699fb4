#!/bin/bash
# Model-level GPU tests (tiny + real shapes) then the headline bench.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
STEPS=${1:-5}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_model_gpu.py tests/test_model_real_shapes_gpu.py > gpurun_out/vb_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/vb_tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps "$STEPS" --warmup 2 > gpurun_out/vb_bench.json 2> gpurun_out/vb_bench.err
rc=$?; cut -c1-900 gpurun_out/vb_bench.json; tail -3 gpurun_out/vb_bench.err; exit $rc
