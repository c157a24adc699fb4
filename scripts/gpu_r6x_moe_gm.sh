#!/bin/bash
# Round 6: MoE variant 4 tile-order row groups (gate_up / down) A/B at T = 16384 / 4096 / 1024,
# interleaved in one process per T; the grouped-GEMM tests (offset clamping included).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${R6X_OUT:-r6x}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "grouped" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for T in 16384 4096 1024; do
  MOE_GM_ARMS="${MOE_GM_ARMS:-4/16,4/4,4/2,8/8,2/8,16/16,8/16}" timeout -k 10 300 python -u scripts/moe_prefill_anatomy.py $T > $O/gm$T.log 2>&1 || { tail -20 $O/gm$T.log; exit 1; }
  grep "^T=" $O/gm$T.log
done
