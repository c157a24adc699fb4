#!/bin/bash
# Round 6: PMC of the MoE layer at Mixtral prefill size (T = 16384): variant 3 (gemm_xd grouped),
# variant 4 (gemm_w4 grouped persistent) and the dense per-expert gemm_w4 arms - MFMA busy,
# wait cycles, L2 hits / misses per GEMM kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6w; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="$R/scripts/moe_prefill_anatomy.py 16384"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS GRBM_GUI_ACTIVE --kernel-include-regex gemm --output-format csv -d $O/p1 -- python3 $ARGS > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --kernel-include-regex gemm --output-format csv -d $O/p3 -- python3 $ARGS > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 1; }
cd $R
python3 scripts/pmc_summary.py $(find $O/p1 -name '*counter_collection.csv') > $O/pmc_p1.txt 2>&1; cat $O/pmc_p1.txt | cut -c1-400
python3 scripts/pmc_summary.py $(find $O/p3 -name '*counter_collection.csv') > $O/pmc_p3.txt 2>&1; cat $O/pmc_p3.txt | cut -c1-400
rm -rf $O/p1 $O/p3
