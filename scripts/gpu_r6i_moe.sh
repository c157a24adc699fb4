#!/bin/bash
# Round 6: Mixtral MoE layer at prefill size - fused MoE vs dense per-expert gemm_w4 GEMMs, and a
# kernel trace of the fused layer (where the time goes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6i; mkdir -p $O
timeout -k 10 300 python -u scripts/moe_prefill_anatomy.py 16384 > $O/anat16k.log 2>&1 || { tail -20 $O/anat16k.log; exit 1; }
grep "^T=" $O/anat16k.log
timeout -k 10 300 python -u scripts/moe_prefill_anatomy.py 4096 > $O/anat4k.log 2>&1 || { tail -20 $O/anat4k.log; exit 1; }
grep "^T=" $O/anat4k.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/scripts/moe_prefill_anatomy.py 16384 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cd $R
S=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats_16k.csv
python3 - "$O/kernel_stats_16k.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms  calls {r["Calls"]:>5}  avg {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
rm -rf $O/prof
