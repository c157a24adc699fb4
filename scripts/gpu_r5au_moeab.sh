#!/bin/bash
# Round 5: Mixtral suggestions wave (batch 1024), router logits read in place by the MoE vs the
# transposed copy (DRTC_ROUTER_VIEW=0), interleaved on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5au; mkdir -p $O
for r in view1 copy1 view2 copy2; do
  v=1; [ "${r#copy}" != "$r" ] && v=0
  DRTC_ROUTER_VIEW=$v timeout -k 10 600 python -u bench.py --model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1 \
    > $O/mix_$r.json 2> $O/mix_$r.err || { tail -5 $O/mix_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/mix_$r.json'));print('$r', d['value'], d.get('p50_latency_ms'))"
done
