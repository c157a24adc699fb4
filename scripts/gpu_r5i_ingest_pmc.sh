#!/bin/bash
# Round 5: PMC passes over the LDS-DMA ingest probe (no MFMA): which unit holds one CU's
# operand stream to ~62-66 GB/s (weights streamed from HBM) / ~90-94 GB/s (cache-resident).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r5i; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
pm() {  # tag, counters [weight source]
  timeout -s KILL 90 rocprofv3 --pmc $2 -d $O/$1 -o pmc --output-format csv -- $R/scripts/native/ingest_probe ${3:-} > $O/$1.log 2>&1
}
pm ah "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" hbm &&
pm ar "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" resident &&
pm a "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" &&
pm b "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_READ_LDS_WAVEFRONTS_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_SERIALIZATION_STALL_sum GRBM_GUI_ACTIVE" &&
pm c "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE" &&
pm d "TCC_BUSY_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_GMI_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE" || { tail -5 $O/*.log; exit 1; }
cd $R
for f in ah ar a b c d; do echo "== $f"; python3 scripts/pmc_summary.py $(find $O/$f -name '*counter_collection.csv'); done > $O/summary.txt
cat $O/summary.txt | cut -c1-400
