#!/bin/bash
# Round 4: PMC comparison of gemm_w4 against hipBLASLt on the prefill shapes (down at
# K = 14336, where the hand kernel loses, and qkv, where it is level): MFMA busy, wait
# buckets, LDS / VMEM instruction counts, L2 hit rate.  One counter pass per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r4j
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
pm() {  # tag, shape, counters
  timeout -s KILL 120 rocprofv3 --pmc $3 -d $R/gpurun_out/r4j/$1 -o pmc --output-format csv -- \
    python3 $R/scripts/w4_probe.py --shape $2 --arms lib,v31 --iters 3 --rounds 2 > $R/gpurun_out/r4j/$1.log 2>&1
}
for sh in 16384,4096,14336 16384,6144,4096; do
  t=$(echo $sh | tr , _)
  pm ${t}_a $sh "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" &&
  pm ${t}_b $sh "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" &&
  pm ${t}_c $sh "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" || exit 1
done
ls -R $R/gpurun_out/r4j | head -40
