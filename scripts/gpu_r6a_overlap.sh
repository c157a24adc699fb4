#!/bin/bash
# Round 6, call 1: the decode-overlap question on one box.
#  1. micro-batched decode numerics (fp32-reference GPU tests)
#  2. hand-written HBM read probe: chip TB/s vs workgroups (CUs) streaming, and the attention's
#     4 KiB random-block access shape
#  3. decode attention at the headline shape with its persistent grid capped
#  4. bench.py interleaved: single-stream decode vs two-stream micro-batched decode (grid caps)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_decode_micro_gpu.py > $O/test_micro.log 2>&1
rc=$?; tail -6 $O/test_micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 scripts/native/stream_probe > $O/stream.log 2>&1 || { tail -5 $O/stream.log; exit 1; }
timeout -k 10 300 python -u scripts/decode_attn_cap.py > $O/attn_cap.log 2>&1 || { tail -20 $O/attn_cap.log; exit 1; }
b() {  # tag, env...
  local tag=$1; shift
  env "$@" DRTC_TIME_DECODE=1 timeout -k 10 240 python -u bench.py --steps 4 --warmup 1 > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  echo "$tag $(python -c "import json,sys;d=json.load(open('$O/bench_$tag.json'));print(d['value'],d['p50_latency_ms'])") $(grep 'decode graph' $O/bench_$tag.err)"
}
b base1 DRTC_DECODE_MICRO=0
b micro1 DRTC_DECODE_MICRO=2
b micro_w128 DRTC_DECODE_MICRO=2 DRTC_DECODE_MICRO_WGS=128
b base2 DRTC_DECODE_MICRO=0
b micro2 DRTC_DECODE_MICRO=2
b micro_nopp DRTC_DECODE_MICRO=2 DRTC_DECODE_MICRO_PINGPONG=0
b micro_w256 DRTC_DECODE_MICRO=2 DRTC_DECODE_MICRO_WGS=256
