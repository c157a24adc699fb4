#!/bin/bash
# Round 5: persistent decode attention with non-temporal K/V loads (DRTC_DECODE_KV_NT=1) vs
# plain: decode-attention GPU tests under NT, the attention micro-bench, then the headline
# interleaved (tokens/s and the engine's decode wall time).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5az; mkdir -p $O
DRTC_DECODE_KV_NT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "paged_decode" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 0 1; do
  DRTC_DECODE_KV_NT=$v timeout -k 10 300 python -u scripts/decode_attn_bench.py 3 llama8b > $O/attn_$v.log 2>&1 || { tail -5 $O/attn_$v.log; exit 1; }
  echo "nt=$v"; grep -A3 "^B1024 ctx150-200" $O/attn_$v.log | tail -1
done
for r in p1 n1 p2 n2; do
  v=0; [ "${r#n}" != "$r" ] && v=1
  DRTC_DECODE_KV_NT=$v timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/$r.json 2> $O/$r.err || { tail -5 $O/$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$r.json'));s=d['engine_stats'];print('$r', d['value'], 'decode_us', s['decode_us'], 'prefill_us', s['prefill_us'])"
done
