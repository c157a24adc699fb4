#!/bin/bash
# Round 3: persistent gemm_w4 (variant 15, cross-tile DMA prefetch) - numerics, then the
# prefill projection shapes against the per-tile form (variant 7) and hipBLASLt.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r3r
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -q --timeout 200 --timeout-method thread -k "w4 or matches_fp32" > gpurun_out/r3r/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3r/tests.log; [ $rc -eq 0 ] || exit $rc
for sh in "16384,6144,4096 store 4" "16384,4096,4096 residual 4" "16384,28672,4096 silu 8" "16384,4096,14336 residual 2" "4400,28672,4096 silu 8" "1024,28672,4096 silu 8"; do
  set -- $sh
  timeout -k 10 120 python -u scripts/w4_probe.py --shape $1 --epi $2 --group-m $3 --arms lib,v7,v15 --iters 10 --rounds 5 >> gpurun_out/r3r/probe.log 2>&1 || exit 1
done
cat gpurun_out/r3r/probe.log
# headline A/B on this box: persistent prefill / decode-GLU gemm_w4 against the per-tile form
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3r/ab_$tag.json 2> gpurun_out/r3r/ab_$tag.err || { tail -5 gpurun_out/r3r/ab_$tag.err; return 1; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/r3r/ab_$tag.json'));print(d['value'],d['ms_per_step'])")"; }
run pers DRTC_W4_PERSIST=1 && run tile DRTC_W4_PERSIST=0 && run pers2 DRTC_W4_PERSIST=1 && run tile2 DRTC_W4_PERSIST=0 || exit 1
# service path, clients -> llm.LLMService over the engine replica: thread-pool vs grpc.aio front-end
svc() {  # tag, args
  local tag=$1; shift
  timeout -k 10 500 python scripts/service_bench.py --model llama-3-8b "$@" > gpurun_out/r3r/service_$tag.json 2> gpurun_out/r3r/service_$tag.err
  local rc=$?; tail -2 gpurun_out/r3r/service_$tag.err; python -c "
import json; d=json.load(open('gpurun_out/r3r/service_$tag.json'))
print('$tag', {k: d.get(k) for k in ('requests','errors','seconds','requests_per_s','gen_tokens_per_s','steady_gen_tokens_per_s','p50_latency_ms','p99_latency_ms')})"; return $rc
}
svc direct_aio --backend pool --client-procs 8 --mode direct --requests 6144 --concurrency 1024 --max-batch 1024 --frontend aio && \
svc direct_threads --backend pool --client-procs 8 --mode direct --requests 6144 --concurrency 1024 --max-batch 1024 --frontend threads
