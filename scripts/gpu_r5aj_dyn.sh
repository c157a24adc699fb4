#!/bin/bash
# Round 5: dynamic item order in the persistent decode attention - numerics (decode tests),
# the attention A/B (dynamic vs static on one box), then a headline pair.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5aj; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "paged_decode" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u scripts/decode_attn_bench.py 3 llama8b > $O/attn.log 2>&1 || { tail -20 $O/attn.log; exit 1; }
grep -v amdgpu $O/attn.log
timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 > $O/bench_dyn.log 2>&1 || { tail -20 $O/bench_dyn.log; exit 1; }
tail -1 $O/bench_dyn.log
DRTC_DECODE_DYN=0 timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 > $O/bench_static.log 2>&1 || { tail -20 $O/bench_static.log; exit 1; }
tail -1 $O/bench_static.log
