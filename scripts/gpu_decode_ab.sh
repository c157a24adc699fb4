#!/bin/bash
# Decode attention variants: numerics, micro-benchmark, end-to-end A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "decode" > gpurun_out/pytest_decode.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_decode.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/decode_attn_bench.py > gpurun_out/decode_attn_bench.log 2>&1
rc=$?; cat gpurun_out/decode_attn_bench.log; [ $rc -ne 0 ] && exit $rc
for v in 1 2; do
  DRTC_DECODE_VARIANT=$v timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_v$v.json 2> gpurun_out/bench_v$v.err
  rc=$?; echo "variant $v"; cut -c1-420 gpurun_out/bench_v$v.json; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python bench.py --model gemma-2b --steps 3 --warmup 1 > gpurun_out/bench_gemma.json 2> gpurun_out/bench_gemma.err
rc=$?; cut -c1-420 gpurun_out/bench_gemma.json; exit $rc
