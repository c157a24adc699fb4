#!/bin/bash
# Headline bench at several prefill chunk sizes (DRTC_PREFILL_CHUNK), alternating, one box;
# then the tuned-GEMM GPU tests.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "tuned" > gpurun_out/tuned_tests.log 2>&1 || { tail -30 gpurun_out/tuned_tests.log; exit 1; }
tail -2 gpurun_out/tuned_tests.log
for i in 1 2; do
  for c in ${CHUNKS:-16384 32768 24576}; do
    DRTC_PREFILL_CHUNK=$c timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
        > gpurun_out/ab_chunk_${c}_$i.json 2> gpurun_out/ab_chunk_${c}_$i.log || exit $?
    echo "chunk=$c run=$i $(python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['p50_ttft_ms'],d['p50_latency_ms'])" gpurun_out/ab_chunk_${c}_$i.json)"
  done
done
