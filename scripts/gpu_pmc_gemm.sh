#!/bin/bash
# PMC counters of the hand-written GEMM (V1 / V5) vs hipBLASLt on one prefill shape.
# Each pass is its own rocprofv3 run (counter limits: 8 SQ, 2 GRBM per pass).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_gemm
mkdir -p $OUT
ARGS="$R/scripts/hgemm_bench.py --model 8b --ms 16384 --only gate_up,qkv --variants 1,5 --splitk 1 --rounds 1 --iters 3 --no-check --out $OUT/b.json"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- python3 $ARGS > $OUT/trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -- python3 $ARGS > $OUT/p1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/p2 -- python3 $ARGS > $OUT/p2.log 2>&1
echo done
