#!/bin/bash
# Round 4: the whole GPU suite, smoke() and the headline bench on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4ai
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r4ai/full_gpu_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r4ai/full_gpu_suite.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4ai/smoke.log 2>&1 || { tail -20 gpurun_out/r4ai/smoke.log; exit 1; }
tail -1 gpurun_out/r4ai/smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/r4ai/bench_default.json 2> gpurun_out/r4ai/bench_default.err || { tail -5 gpurun_out/r4ai/bench_default.err; exit 1; }
cut -c1-200 gpurun_out/r4ai/bench_default.json
