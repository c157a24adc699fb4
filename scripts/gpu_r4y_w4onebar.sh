#!/bin/bash
# Round 4: gemm_w4 with one barrier fewer per K tile (variants 111 / 127): fp32 tests, then
# interleaved A/B against 63 and the library on the prefill shapes and the decode gate_up + GLU,
# then the headline with 127 vs 63.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4y
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py -k "persistent or mfma_gemm" > gpurun_out/r4y/tests.log 2>&1 || { tail -30 gpurun_out/r4y/tests.log; exit 1; }
tail -1 gpurun_out/r4y/tests.log
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 10 --rounds 5"
{
$P --shape 16384,6144,4096 --arms lib,v63,v127,v47,v111 --group-m 4 &&
$P --shape 16384,4096,4096 --epi residual --arms lib,v63,v127 --group-m 4 &&
$P --shape 16384,28672,4096 --epi silu --arms lib,v63,v127 &&
$P --shape 16384,4096,14336 --arms lib,v63,v127 --group-m 2 &&
$P --shape 1024,28672,4096 --epi silu --arms lib,v63,v127 --rotate 3
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4y/probe.log || exit 1
b() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4y/bench_$tag.json 2> gpurun_out/r4y/bench_$tag.err || { tail -5 gpurun_out/r4y/bench_$tag.err; return 1; }
  echo $tag $(cut -c1-120 gpurun_out/r4y/bench_$tag.json)
}
b v127 DRTC_W4_VARIANT=127 && b v63 DRTC_W4_VARIANT=63 && b v127b DRTC_W4_VARIANT=127
