#!/bin/bash
# Round 4: gemm_xd with non-temporal weight loads (forms + 1000) on the decode shapes whose batch
# fits one row tile: fp32 tests, interleaved A/B against the plain forms (Llama-3-70B and
# Llama-3-8B at M = 128-256), then the 70B ask-AI wave at batch 256 with and without.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4aa
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py -k "xd" > gpurun_out/r4aa/tests.log 2>&1 || { tail -30 gpurun_out/r4aa/tests.log; exit 1; }
tail -1 gpurun_out/r4aa/tests.log
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
{
$P --shape 256,8192,28672 --arms lib,x244,x1244,x284,x1284 --rotate 2 &&
$P --shape 256,57344,8192 --epi silu --arms x241,x1241,x281,x1281 --rotate 2 &&
$P --shape 256,8192,8192 --arms lib,x244,x1244,x242,x1242 --rotate 4 &&
$P --shape 256,10240,8192 --arms lib,x241,x1241,x242,x1242 --rotate 4 &&
$P --shape 128,8192,28672 --arms lib,x144,x1144,x148,x1148 --rotate 2 &&
$P --shape 256,28672,4096 --epi silu --arms x241,x1241 --rotate 3 &&
$P --shape 256,4096,14336 --arms lib,x244,x1244 --rotate 4
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4aa/probe.log || exit 1
for nt in 1 0; do
  DRTC_XD_NT=$nt timeout -k 10 600 python -u bench.py --model llama-3-70b --workload ask --batch 256 --steps 3 --warmup 1 \
    > gpurun_out/r4aa/b70_nt$nt.json 2> gpurun_out/r4aa/b70_nt$nt.err || { tail -5 gpurun_out/r4aa/b70_nt$nt.err; exit 1; }
  cut -c1-400 gpurun_out/r4aa/b70_nt$nt.json
done
