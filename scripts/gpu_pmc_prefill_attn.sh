#!/bin/bash
# PMC counters of the prefill attention kernel on the smart-reply batch shape.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 --list-avail > "$R/gpurun_out/pmc_avail.txt" 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA --kernel-include-regex prefill_attn --output-format csv -d "$R/gpurun_out/pmc_pa" -o run -- python3 "$R/scripts/prefill_attn_bench.py" --only llama8b_smart_reply > "$R/gpurun_out/pmc_pa.log" 2>&1
echo "pmc rc=$?"
