#!/bin/bash
# Round 3: RMSNorm folded across prefill layers (o / down epilogue row statistic, qkv /
# gate_up scale their rows) - numerics, then a headline A/B on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py tests/test_model_real_shapes_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/t_r3m.log 2>&1
rc=$?; tail -4 gpurun_out/t_r3m.log; [ $rc -le 1 ] || exit $rc
run() { local tag=$1; shift; env "$@" timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -5 gpurun_out/ab_$tag.err; return 1; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print(d['value'],d['ms_per_step'])")"; }
run fold DRTC_FOLD_NORM=1 && run nofold DRTC_FOLD_NORM=0 && run fold2 DRTC_FOLD_NORM=1 && run nofold2 DRTC_FOLD_NORM=0
