#!/bin/bash
# Round 3: folded RMSNorm with temporal stores for the residual stream (stays in the MALL for
# the consumer GEMM) - A/B on one box; the residual-epilogue model test.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_gemm_gpu.py -q --timeout 200 --timeout-method thread -k "residual or rinv or rs_linear or folded" > gpurun_out/t_r3n.log 2>&1
rc=$?; tail -3 gpurun_out/t_r3n.log; [ $rc -le 1 ] || exit $rc
run() { local tag=$1; shift; env "$@" timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -5 gpurun_out/ab_$tag.err; return 1; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print(d['value'],d['ms_per_step'])")"; }
run fold DRTC_FOLD_NORM=1 && run nofold DRTC_FOLD_NORM=0 && run fold2 DRTC_FOLD_NORM=1 && run nofold2 DRTC_FOLD_NORM=0
