#!/bin/bash
# Full GPU validation + headline bench (3 steps) + Llama-3-8B summarize bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
rc=$?; cut -c1-700 gpurun_out/bench_final.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py --workload summarize --batch 512 --steps 2 > gpurun_out/bench_summarize.json 2> gpurun_out/bench_summarize.err
rc=$?; cut -c1-600 gpurun_out/bench_summarize.json; exit $rc
