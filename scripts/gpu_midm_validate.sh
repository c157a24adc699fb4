#!/bin/bash
# Medium-M GEMM tests, model tests (decode graphs now take it for tuned shapes), and the
# small-batch decode benches with it on / off.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gemm_gpu.py -k midm > gpurun_out/mv_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_model_gpu.py tests/test_model_real_shapes_gpu.py > gpurun_out/mv_model.log 2>&1
rc=$?; tail -3 gpurun_out/mv_model.log; [ $rc -eq 0 ] || exit $rc
for B in 32 64 128; do
  for M in 1 0; do
    DRTC_MIDM_GEMM=$M timeout -k 10 300 python -u bench.py --batch $B --steps 5 --warmup 2 \
      > gpurun_out/mv_b${B}_m$M.json 2> gpurun_out/mv_b${B}_m$M.err || { echo "bench B=$B midm=$M failed"; tail -5 gpurun_out/mv_b${B}_m$M.err; exit 1; }
    python -c "import json,sys; r=json.loads(open('gpurun_out/mv_b${B}_m$M.json').read().splitlines()[-1]); print('B=$B midm=$M', r['value'], 'tok/s p50', r['p50_latency_ms'])"
  done
done
