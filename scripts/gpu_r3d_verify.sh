#!/bin/bash
# Round 3 re-verification: the whole GPU suite (no -x: every failure listed in one call; an
# assertion failure is not a GPU fault, anything else - abort, segfault, timeout - ends the
# call), smoke(), then a 10-step headline bench.
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/full_gpu_suite.log 2>&1
rc=$?; tail -15 gpurun_out/full_gpu_suite.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_r3d.json 2> gpurun_out/bench_r3d.err || { tail -20 gpurun_out/bench_r3d.err; exit 1; }
cat gpurun_out/bench_r3d.json
