#!/bin/bash
# Round 5: headline with the RMSNorm store forms interleaved (DRTC_NORM_VARIANT 0 plain / 1
# non-temporal): tokens/s and the engine's decode wall time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5ay; mkdir -p $O
for r in p1 n1 p2 n2; do
  v=0; [ "${r#n}" != "$r" ] && v=1
  DRTC_NORM_VARIANT=$v timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/$r.json 2> $O/$r.err || { tail -5 $O/$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$r.json'));s=d['engine_stats'];print('$r', d['value'], 'decode_us', s['decode_us'], 'prefill_us', s['prefill_us'])"
done
