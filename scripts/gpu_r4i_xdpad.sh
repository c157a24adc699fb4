#!/bin/bash
# Round 4: gemm_xd forms (128/256-row tiles, split-K 2) - fp32 tests, A/B against the tuned
# library at the decode shapes, operand row-stride padding probe, PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r4i
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py -k "xd" > gpurun_out/r4i/tests.log 2>&1 || { tail -30 gpurun_out/r4i/tests.log; exit 1; }
tail -2 gpurun_out/r4i/tests.log
P="timeout -k 10 120 python -u scripts/w4_probe.py --iters 20 --rounds 7"
{
$P --shape 1024,4096,4096 --arms lib,x141,x241,x242 --rotate 10 &&
$P --shape 1024,6144,4096 --arms lib,x161,x261,x262,x242 --rotate 8 &&
$P --shape 1024,4096,14336 --arms lib,x141,x241,x242 --rotate 4 &&
$P --shape 768,4096,4096 --arms lib,x141,x242 --rotate 10 &&
$P --shape 768,6144,4096 --arms lib,x161,x262,x242 --rotate 8 &&
$P --shape 768,4096,14336 --arms lib,x141,x242 --rotate 4 &&
$P --shape 512,4096,4096 --arms lib,x121,x242 --rotate 10 &&
$P --shape 512,6144,4096 --arms lib,x121,x242,x262 --rotate 8 &&
$P --shape 512,4096,14336 --arms lib,x121,x242 --rotate 4 &&
$P --shape 256,8192,28672 --arms lib,x121,x242 --rotate 2 &&
$P --shape 256,8192,8192 --arms lib,x121,x242 --rotate 4
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4i/probe.log || exit 1
timeout -k 10 120 python -u scripts/xd_pad_probe.py --shape 1024,4096,4096 --nf 4 --pads 0,64,256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4i/pad.log || exit 1
cd /tmp && export TMPDIR=/tmp
pm() {  # tag, counters
  timeout -s KILL 90 rocprofv3 --pmc $2 -d $R/gpurun_out/r4i/pmc_$1 -o pmc --output-format csv -- \
    python3 $R/scripts/w4_probe.py --shape 1024,4096,4096 --arms lib,x141,x242 --rotate 10 --iters 5 --rounds 2 > /dev/null 2>&1
}
pm a "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" &&
pm b "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" &&
pm c "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
ls -R $R/gpurun_out/r4i | head -30
