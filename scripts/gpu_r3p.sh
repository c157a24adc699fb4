#!/bin/bash
# Round 3: fused decode RoPE with the step position read one item ahead - tests, then
# headline A/B (fused vs two launches) on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q --timeout 200 --timeout-method thread -k "fused_rope or decode or graph" > gpurun_out/t_r3p.log 2>&1
rc=$?; tail -3 gpurun_out/t_r3p.log; [ $rc -le 1 ] || exit $rc
run() { local tag=$1; shift; env "$@" timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -5 gpurun_out/ab_$tag.err; return 1; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print(d['value'],d['ms_per_step'])")"; }
run fused DRTC_DECODE_FUSED_ROPE=1 && run unfused DRTC_DECODE_FUSED_ROPE=0 && run fused2 DRTC_DECODE_FUSED_ROPE=1 && run unfused2 DRTC_DECODE_FUSED_ROPE=0
