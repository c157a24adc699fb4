#!/bin/bash
# Round 6: the decode attention kernel without the loop-entry waitcnt merge stall (first block
# landed before the block loop) vs the round-5 form, interleaved: kernel alone at the headline
# shape, the decode-attention GPU tests, and the headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "decode or paged" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for pw in 0 1; do
    DRTC_DECODE_PREWAIT=$pw timeout -k 10 200 python -u scripts/decode_attn_cap.py 0,256 > $O/attn_pw${pw}_$i.log 2>&1 || { tail -5 $O/attn_pw${pw}_$i.log; exit 1; }
    echo "prewait=$pw run $i: $(grep '"max_wgs": 0' $O/attn_pw${pw}_$i.log | tr '\n' ' ')"
  done
done
for i in 1 2; do
  for pw in 0 1; do
    DRTC_DECODE_PREWAIT=$pw DRTC_TIME_DECODE=1 timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 > $O/bench_pw${pw}_$i.json 2> $O/bench_pw${pw}_$i.err || { tail -20 $O/bench_pw${pw}_$i.err; exit 1; }
    echo "bench prewait=$pw run $i: $(python -c "import json;d=json.load(open('$O/bench_pw${pw}_$i.json'));print(d['value'],d['p50_latency_ms'])") $(grep 'decode graph' $O/bench_pw${pw}_$i.err)"
  done
done
