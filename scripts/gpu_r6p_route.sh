#!/bin/bash
# Round 6: three-pass MoE routing (multi-workgroup top-k + stable scatter) - tests, the layer at
# prefill and decode size with a kernel trace, the Mixtral waves.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6p; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py -k "grouped or moe" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for T in 16384 1024; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$T -o run -- python3 $R/scripts/moe_prefill_anatomy.py $T > $O/anat$T.log 2>&1 || { tail -5 $O/anat$T.log; exit 1; }
  S=$(find $O/prof$T -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats_$T.csv; rm -rf $O/prof$T
  grep "^T=" $O/anat$T.log
  python3 - "$O/kernel_stats_$T.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms  calls {r["Calls"]:>5}  avg {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:100]}')
PY
done
cd $R
bash scripts/gpu_r6h_configs.sh r6p mix_1024a "--model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1" \
  mix_1024b "--model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1" \
  mix_256 "--model mixtral-8x7b --workload suggest --batch 256 --steps 3 --warmup 1" || exit 1
