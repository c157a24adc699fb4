#!/bin/bash
# Round 4: the whole GPU suite and smoke() after the non-temporal gemm_xd forms, then the
# non-temporal forms probed at the headline's M = 1024 (8 row tiles share each weight panel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4ac
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r4ac/full_gpu_suite.log 2>&1
rc=$?; tail -5 gpurun_out/r4ac/full_gpu_suite.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4ac/smoke.log 2>&1 || { tail -20 gpurun_out/r4ac/smoke.log; exit 1; }
tail -1 gpurun_out/r4ac/smoke.log
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
{
$P --shape 1024,6144,4096 --arms lib,x161,x1161 --rotate 8 &&
$P --shape 1024,4096,4096 --arms lib,x141,x1141 --rotate 10 &&
$P --shape 1024,4096,14336 --arms lib,x242,x1242 --rotate 4 &&
$P --shape 1024,28672,4096 --epi silu --arms x281,x1281 --rotate 3
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4ac/probe.log
