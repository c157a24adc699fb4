#!/bin/bash
# Round 4: gemm_xd operand row-stride padding probe + PMC pass (L2 hit / requests / waits).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4i
export HSA_ENABLE_IPC_MODE_LEGACY=0
P="timeout -k 10 120 python -u scripts/xd_pad_probe.py"
{
$P --shape 1024,4096,4096 --nf 4 --pads 0,64,128,256,512 &&
$P --shape 1024,4096,14336 --nf 4 --pads 0,64,128 --rotate 4 &&
$P --shape 1024,6144,4096 --nf 6 --pads 0,64,128 --rotate 8
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4i/pad.log || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
pm() {  # tag, counters
  timeout -s KILL 90 rocprofv3 --pmc $2 -d $R/gpurun_out/r4i/pmc_$1 -o pmc --output-format csv -- \
    python3 $R/scripts/w4_probe.py --shape 1024,4096,4096 --arms lib,x4 --rotate 10 --iters 5 --rounds 2 > /dev/null 2>&1
}
pm a "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" &&
pm b "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" &&
pm c "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES TA_BUSY_avr TA_TA_BUSY_sum"
ls -R $R/gpurun_out/r4i | head -30
