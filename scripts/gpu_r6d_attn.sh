#!/bin/bash
# Round 6: decode attention with the step token's k / v / cos-sin rows staged into LDS one item
# ahead (fused RoPE path) - numerics, kernel time vs the two-launch form (rope_kv + plain
# persistent attention, DRTC_DECODE_FUSED_ROPE=0), headline A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_decode_micro_gpu.py tests/test_model_gpu.py tests/test_model_real_shapes_gpu.py -k "decode or paged or rope or micro or serving or engine or graph or mixed" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for fr in 1 0; do
    DRTC_DECODE_FUSED_ROPE=$fr timeout -k 10 200 python -u scripts/decode_attn_cap.py 0 > $O/attn_fr${fr}_$i.log 2>&1 || { tail -5 $O/attn_fr${fr}_$i.log; exit 1; }
    echo "fused_rope=$fr run $i: $(grep -v amdgpu $O/attn_fr${fr}_$i.log | tr '\n' ' ')"
  done
done
for i in 1 2; do
  for fr in 1 0; do
    DRTC_DECODE_FUSED_ROPE=$fr DRTC_TIME_DECODE=1 timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 > $O/bench_fr${fr}_$i.json 2> $O/bench_fr${fr}_$i.err || { tail -20 $O/bench_fr${fr}_$i.err; exit 1; }
    echo "bench fused_rope=$fr run $i: $(python -c "import json;d=json.load(open('$O/bench_fr${fr}_$i.json'));print(d['value'],d['p50_latency_ms'])") $(grep 'decode graph' $O/bench_fr${fr}_$i.err)"
  done
done
