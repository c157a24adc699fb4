#!/bin/bash
# Round 5: 70B ask wave (batch 256, ~34.8k prompt tokens): the 2.8k-token last prefill chunk on gemm_w4
# (DRTC_W4_MIN_M=2048) vs on the library (default 4096), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5bf; mkdir -p $O
for r in d1 c1 d2 c2; do
  ch=4096; [ "${r#c}" != "$r" ] && ch=2048
  DRTC_W4_MIN_M=$ch timeout -k 10 500 python -u bench.py --model llama-3-70b --workload ask --batch 256 --steps 3 --warmup 1 \
    > $O/$r.json 2> $O/$r.err || { tail -5 $O/$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$r.json'));s=d['engine_stats'];print('$r w4_min_m $ch', d['value'], 'p50', d['p50_latency_ms'], 'ttft', d['p50_ttft_ms'], 'prefill_steps', s['prefill_steps'], 'prefill_us', s['prefill_us'])"
done
