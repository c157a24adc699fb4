#!/bin/bash
# Round 6: same-box A/B of the V-cache slot-row layout: ab_old/ (the previous [8][D][4] layout,
# built in-tree from HEAD sources) vs the working tree, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6ab; mkdir -p $O
for r in 1 2; do
  for arm in old new; do
    D=$R; [ $arm = old ] && D=$R/ab_old
    (cd $D && timeout -k 10 300 python -u scripts/decode_attn_cap.py 0 sorted > $O/attn_${arm}_$r.log 2>&1) || { tail -5 $O/attn_${arm}_$r.log; exit 1; }
    echo "$arm $r $(grep '"B"' $O/attn_${arm}_$r.log | tr '\n' ' ')"
    (cd $D && timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/bench_${arm}_$r.json 2> $O/bench_${arm}_$r.err) || { tail -5 $O/bench_${arm}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${arm}_$r.json'));print('$arm', $r, d['value'], d['p50_latency_ms'], d['engine_stats'].get('decode_us'), d['engine_stats'].get('decode_steps'))"
  done
done
