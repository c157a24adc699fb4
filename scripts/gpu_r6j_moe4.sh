#!/bin/bash
# Round 6: MoE variant 4 (expert-ordered rows + gemm_w4 grouped persistent GEMMs) - tests, the
# layer at prefill size against variant 3 / dense, a kernel trace, and the Mixtral wave A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6j; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py -k "grouped or moe" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/moe_prefill_anatomy.py 16384 > $O/anat16k.log 2>&1 || { tail -20 $O/anat16k.log; exit 1; }
grep "^T=" $O/anat16k.log
DRTC_MOE_CHUNK=16384 timeout -k 10 300 python -u scripts/moe_prefill_anatomy.py 16384 > $O/anat16k_c16.log 2>&1 || { tail -20 $O/anat16k_c16.log; exit 1; }
grep "^T=" $O/anat16k_c16.log
timeout -k 10 300 python -u scripts/moe_prefill_anatomy.py 4096 > $O/anat4k.log 2>&1 || { tail -20 $O/anat4k.log; exit 1; }
grep "^T=" $O/anat4k.log
timeout -k 10 400 python -u scripts/moe_bench.py 14336 1024,2048,4096 > $O/moe_bench.log 2>&1 || { tail -20 $O/moe_bench.log; exit 1; }
grep "^T=" $O/moe_bench.log | cut -c1-400
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
bash scripts/gpu_r6h_configs.sh r6j mix_auto "--model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1" || exit 1
DRTC_MOE_VARIANT=3 bash scripts/gpu_r6h_configs.sh r6j mix_v3 "--model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1" || exit 1
DRTC_MOE_CHUNK=16384 bash scripts/gpu_r6h_configs.sh r6j mix_auto_c16 "--model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1" || exit 1
