#!/bin/bash
# Round 3 A/B on one box: headline with the fused decode RoPE + register sampler (default)
# vs the two-launch RoPE, vs the streaming sampler; sampler timing of both paths.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k "sample or fused_rope" > gpurun_out/t_ab.log 2>&1 || { tail -30 gpurun_out/t_ab.log; exit 1; }
tail -1 gpurun_out/t_ab.log
for v in 1 0; do
  DRTC_SAMPLE_REG=$v timeout -k 10 200 python -u scripts/sampler_bench.py --rounds 3 > gpurun_out/sampler_reg$v.log 2>&1 || exit 1
  grep -v amdgpu gpurun_out/sampler_reg$v.log | grep randn_s2 | sed "s/^/reg=$v /"
done
run() { local tag=$1; shift; env "$@" timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -5 gpurun_out/ab_$tag.err; return 1; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print(d['value'],d['ms_per_step'])")"; }
run fused DRTC_DECODE_FUSED_ROPE=1 && run unfused DRTC_DECODE_FUSED_ROPE=0 && run fused2 DRTC_DECODE_FUSED_ROPE=1 && run streamsamp DRTC_SAMPLE_REG=0
