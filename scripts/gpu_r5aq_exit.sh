#!/bin/bash
# Round 5: find what aborts the GPU test process at interpreter exit ("terminate called
# without an active exception" after every test passed): faulthandler on, threads listed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5aq; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DRTC_TEST_THREADS=1
timeout -k 10 900 python -X faulthandler -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/gpu_suite.log 2>&1
rc=$?; tail -40 $O/gpu_suite.log; exit $rc
