#!/bin/bash
# Round 4: decode-shape (M = 1024) gemm_w4 split-K with the K-slice-by-XCD tile order
# (group_m < 0) vs the tile-major order and the tuned library, weights streamed from HBM;
# then L2 hit counters for the o projection arms.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r4a
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4a
: > $O/probe.log
for spec in "1024,4096,4096 store 10 lib,v7:4:4,v7:4:-4,v11:4:4,v11:4:-4,v11:4:-2" \
            "1024,4096,14336 store 4 lib,v7:4:4,v7:4:-4,v11:4:4,v11:4:-4,v11:4:-2" \
            "1024,6144,4096 store 8 lib,v7:2:4,v7:2:-4,v11:2:4,v11:2:-4" \
            "512,4096,4096 store 10 lib,v7:4:-2,v11:4:-2,v7:8:-2" \
            "768,4096,4096 store 10 lib,v7:4:-4,v11:4:-4"; do
  set -- $spec
  timeout -k 10 200 python -u scripts/w4_probe.py --shape $1 --epi $2 --rotate $3 --arms $4 --iters 20 >> $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
done
grep -v amdgpu $O/probe.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for arm in lib v11:4:4 v11:4:-4; do
  t=$(echo $arm | tr ':' '_')
  ARGS="$R/scripts/w4_probe.py --shape 1024,4096,4096 --rotate 10 --arms $arm --rounds 1 --iters 3"
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d $R/$O/p3_$t -- python3 $ARGS > $R/$O/p3_$t.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $R/$O/p1_$t -- python3 $ARGS > $R/$O/p1_$t.log 2>&1 || exit 1
  echo "#### $arm" >> $R/$O/pmc.txt
  python3 $R/scripts/pmc_summary.py $R/$O/p3_$t $R/$O/p1_$t | grep -A20 "w4\|hipblaslt" >> $R/$O/pmc.txt
done
cat $R/$O/pmc.txt
