#!/bin/bash
# Round 4: gemm_xd 256x256 probes, 70B ask-AI at batch 256 / 224 with the xd decode GEMMs,
# and the service path with the serving defaults (direct and via the Raft leader).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4p
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
{
$P --shape 1024,28672,4096 --epi silu --arms lib,v31,x281,x241 --rotate 3 &&
$P --shape 768,28672,4096 --epi silu --arms lib,v31,x281 --rotate 3 &&
$P --shape 512,28672,4096 --epi silu --arms lib,v31,x281,x241 --rotate 3 &&
$P --shape 1024,4096,14336 --arms lib,x242,x282,x284 --rotate 4 &&
$P --shape 256,8192,28672 --arms lib,x244,x284,x288 --rotate 2 &&
$P --shape 256,57344,8192 --epi silu --arms lib,x241,x281 --rotate 2 &&
$P --shape 256,8192,8192 --arms lib,x121,x284,x282 --rotate 4 &&
$P --shape 16384,6144,4096 --arms lib,v31,x281 --rotate 1
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4p/probe.log || exit 1
for b in 256 224; do
  timeout -k 10 600 python -u bench.py --model llama-3-70b --workload ask --batch $b --steps 3 --warmup 1 \
    > gpurun_out/r4p/b70_$b.json 2> gpurun_out/r4p/b70_$b.err || { tail -5 gpurun_out/r4p/b70_$b.err; exit 1; }
  cut -c1-400 gpurun_out/r4p/b70_$b.json
done
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r4p/engine.json 2> gpurun_out/r4p/engine.err || exit 1
cut -c1-120 gpurun_out/r4p/engine.json
for m in direct raft; do
  timeout -k 10 500 python scripts/service_bench.py --model llama-3-8b --backend pool --client-procs 8 \
    --requests 10240 --concurrency 1024 --max-batch 1024 --mode $m > gpurun_out/r4p/service_$m.json 2> gpurun_out/r4p/service_$m.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/r4p/service_$m.json'))
print('$m', {k: d.get(k) for k in ('requests','errors','seconds','gen_tokens_per_s','p50_latency_ms','p99_latency_ms')}, d.get('replica_delta'))"
done
