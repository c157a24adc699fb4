#!/bin/bash
# Round 4 final tree: kernel-trace anatomy of the headline, the whole GPU suite, smoke(), and
# a 10-step headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_prof_model.sh r4z --steps 2 --warmup 1 > gpurun_out/prof_r4z.out 2>&1
rc=$?; tail -3 gpurun_out/prof_r4z.out; [ $rc -eq 0 ] || exit $rc
python scripts/trace_gaps.py gpurun_out/r4z_kernel_trace.csv.gz > gpurun_out/r4z_gaps.txt 2>&1 || true
head -3 gpurun_out/r4z_gaps.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/full_gpu_suite.log 2>&1
rc=$?; tail -5 gpurun_out/full_gpu_suite.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_r4z.json 2> gpurun_out/bench_r4z.err || { tail -20 gpurun_out/bench_r4z.err; exit 1; }
cut -c1-200 gpurun_out/bench_r4z.json
