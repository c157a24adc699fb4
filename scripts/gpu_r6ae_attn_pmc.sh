#!/bin/bash
# Round 6 (counters): the fused-RoPE persistent decode attention at the
# headline shape (B = 1024, contexts 150-200) on the full grid and capped at 128 / 64
# workgroups - HBM read requests, L2 hits / misses, wait vs active cycles per dispatch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6ae; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cap in 0 128 64; do
  cd $R
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --kernel-include-regex paged_decode --output-format csv -d $O/m$cap -- python3 scripts/decode_attn_cap.py $cap sorted > $O/m$cap.log 2>&1 || { tail -5 $O/m$cap.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-include-regex paged_decode --output-format csv -d $O/s$cap -- python3 scripts/decode_attn_cap.py $cap sorted > $O/s$cap.log 2>&1 || { tail -5 $O/s$cap.log; exit 1; }
  echo "cap $cap: $(grep '"B": 1024' $O/m$cap.log)"
  python3 scripts/pmc_summary.py $(find $O/m$cap -name '*counter_collection.csv') > $O/pmc_mem_$cap.txt
  python3 scripts/pmc_summary.py $(find $O/s$cap -name '*counter_collection.csv') > $O/pmc_sq_$cap.txt
  cut -c1-400 $O/pmc_mem_$cap.txt $O/pmc_sq_$cap.txt
  rm -rf $O/m$cap $O/s$cap
done
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k moe > $O/moe_tests.log 2>&1 || { tail -5 $O/moe_tests.log; exit 1; }
tail -1 $O/moe_tests.log
