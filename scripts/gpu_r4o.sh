#!/bin/bash
# Round 4: gemm_xd 256x256 forms (tests, decode gate_up + GLU vs gemm_w4, 70B M = 256
# shapes, a prefill shape), then the closed-loop service with arrival gathering.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_service_gpu.py -k "xd or norm_glu or side_by_side" > gpurun_out/r4o/tests.log 2>&1 || { tail -30 gpurun_out/r4o/tests.log; exit 1; }
tail -1 gpurun_out/r4o/tests.log
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
{
$P --shape 1024,28672,4096 --epi silu --arms lib,v31,x281,x282,x241 --rotate 3 &&
$P --shape 768,28672,4096 --epi silu --arms lib,v31,x281,x241 --rotate 3 &&
$P --shape 512,28672,4096 --epi silu --arms lib,v31,x281,x241 --rotate 3 &&
$P --shape 1024,4096,14336 --arms lib,x242,x282,x284 --rotate 4 &&
$P --shape 1024,4096,4096 --arms lib,x141,x282 --rotate 10 &&
$P --shape 256,8192,28672 --arms lib,x244,x284,x288 --rotate 2 &&
$P --shape 256,57344,8192 --epi silu --arms lib,x241,x281 --rotate 2 &&
$P --shape 256,8192,8192 --arms lib,x121,x284,x282 --rotate 4 &&
$P --shape 256,10240,8192 --arms lib,x243,x284 --rotate 4 &&
$P --shape 16384,6144,4096 --arms lib,v31,x281 --rotate 1
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4o/probe.log || exit 1
svc() {  # tag, args
  local tag=$1; shift
  env "$@" timeout -k 10 500 python scripts/service_bench.py --model llama-3-8b --backend pool --client-procs 8 \
    --requests 10240 --concurrency 1024 --max-batch 1024 $MODE > gpurun_out/r4o/service_$tag.json 2> gpurun_out/r4o/service_$tag.err
  local rc=$?; python -c "
import json; d=json.load(open('gpurun_out/r4o/service_$tag.json'))
print('$tag', {k: d.get(k) for k in ('requests','errors','seconds','gen_tokens_per_s','p50_latency_ms','p99_latency_ms')}, d.get('replica_delta'))"; return $rc
}
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r4o/engine.json 2> gpurun_out/r4o/engine.err || exit 1
cut -c1-120 gpurun_out/r4o/engine.json
MODE="--mode direct"
svc g3 DRTC_BURST_GAP_MS=3 && svc g3_a16k DRTC_BURST_GAP_MS=3 DRTC_ADMIT_MIN_TOKENS=16384 && \
svc g3_a8k DRTC_BURST_GAP_MS=3 DRTC_ADMIT_MIN_TOKENS=8192 || exit 1
MODE="--mode raft"
svc raft_g3 DRTC_BURST_GAP_MS=3 && svc raft_g3_a16k DRTC_BURST_GAP_MS=3 DRTC_ADMIT_MIN_TOKENS=16384
