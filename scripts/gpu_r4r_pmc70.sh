#!/bin/bash
# Round 4: PMC of gemm_xd on the Llama-3-70B M = 256 down shape (256x128 x 4 slices) against
# the library: is the weight stream latency- or L2-bound?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r4r
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
pm() {  # tag, counters
  timeout -s KILL 120 rocprofv3 --pmc $2 -d $R/gpurun_out/r4r/$1 -o pmc --output-format csv -- \
    python3 $R/scripts/w4_probe.py --shape 256,8192,28672 --arms lib,x244,x121 --rotate 2 --iters 5 --rounds 2 > $R/gpurun_out/r4r/$1.log 2>&1
}
pm a "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" &&
pm b "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" &&
pm c "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum GRBM_GUI_ACTIVE"
cd $R
for p in a b c; do echo "== $p"; python scripts/pmc_summary.py gpurun_out/r4r/$p/pmc_counter_collection.csv | grep -v "void at::\|elementwise\|rocclr\|S_B_Bias_HA_S_SAV_UserArg"; done
