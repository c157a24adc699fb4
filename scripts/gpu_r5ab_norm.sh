#!/bin/bash
# Round 5: RMSNorm weight prefetch A/B (DRTC_NORM_NOPF=1: the weight row loaded after the
# reduction, as before) at decode sizes, plus the norm fp32 tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "norm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  DRTC_NORM_NOPF=1 timeout -k 10 120 python -u scripts/norm_probe.py > $O/nopf_$r.log 2>&1 || { tail -5 $O/nopf_$r.log; exit 1; }
  timeout -k 10 120 python -u scripts/norm_probe.py > $O/pf_$r.log 2>&1 || { tail -5 $O/pf_$r.log; exit 1; }
done
paste <(grep '^{' $O/nopf_2.log | cut -c1-70) <(grep '^{' $O/pf_2.log | python3 -c "import sys,json;[print(json.loads(l)['us']) for l in sys.stdin]")
