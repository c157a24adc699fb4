#!/bin/bash
# Round 3: split-K partial planes summed in the next RMSNorm (decode o / down) - numerics,
# then a headline A/B on one box; sampler tail (rank-count sort + block scan) tests + timing.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -q --timeout 200 --timeout-method thread -k "partials or sample" > gpurun_out/t_r3j.log 2>&1
rc=$?; tail -3 gpurun_out/t_r3j.log; [ $rc -le 1 ] || exit $rc  # assertion failures: keep going
timeout -k 10 200 python -u scripts/sampler_bench.py --rounds 3 > gpurun_out/sampler_bench.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/sampler_bench.log | grep randn_s2
run() { local tag=$1; shift; env "$@" timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -5 gpurun_out/ab_$tag.err; return 1; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print(d['value'],d['ms_per_step'])")"; }
run base DRTC_W4_PARTIAL= && run down DRTC_W4_PARTIAL=4096:14336:4 && run down_o DRTC_W4_PARTIAL=4096:14336:4,4096:4096:4 && run base2 DRTC_W4_PARTIAL=
