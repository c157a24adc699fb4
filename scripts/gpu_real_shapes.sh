#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_model_real_shapes_gpu.py > gpurun_out/real_shapes.log 2>&1
rc=$?; tail -15 gpurun_out/real_shapes.log; exit $rc
