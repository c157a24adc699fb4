#!/bin/bash
# Round 5: PMC comparison gemm_ring vs gemm_w4 v63 vs hipBLASLt on the prefill down shape
# (K = 14336) and qkv: wait buckets, MFMA busy, LDS, L2 requests.  One counter pass per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r5c; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
pm() {  # tag, shape, group_m, counters
  timeout -s KILL 120 rocprofv3 --pmc $4 -d $O/$1 -o pmc --output-format csv -- \
    python3 $R/scripts/w4_probe.py --shape $2 --arms lib,v63,r$3 --group-m $3 --iters 3 --rounds 2 > $O/$1.log 2>&1
}
for sg in 16384,4096,14336:2 16384,6144,4096:4; do
  sh=${sg%%:*}; gm=${sg##*:}
  t=$(echo $sh | tr , _)
  pm ${t}_a $sh $gm "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" &&
  pm ${t}_b $sh $gm "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" &&
  pm ${t}_c $sh $gm "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" || exit 1
done
cd $R
for f in $(ls -d $O/*_a $O/*_b $O/*_c); do echo "== $(basename $f)"; python3 scripts/pmc_summary.py $(find $f -name '*counter_collection.csv'); done > $O/summary.txt
cat $O/summary.txt
