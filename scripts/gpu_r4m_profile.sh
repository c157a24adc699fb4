#!/bin/bash
# Round 4: kernel-trace profile of the headline (per-phase anatomy, decode busy per step)
# with gemm_xd on the decode path, then the whole GPU suite and smoke().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_prof_model.sh r4m --steps 2 --warmup 1 > gpurun_out/prof_r4m.out 2>&1
rc=$?; tail -3 gpurun_out/prof_r4m.out; [ $rc -eq 0 ] || exit $rc
python scripts/trace_gaps.py gpurun_out/r4m_kernel_trace.csv.gz > gpurun_out/r4m_gaps.txt 2>&1 || true
head -3 gpurun_out/r4m_gaps.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/full_gpu_suite.log 2>&1
rc=$?; tail -15 gpurun_out/full_gpu_suite.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
