#!/bin/bash
# Round 5: gemm_w4 persistent form with temporal epilogue stores (DRTC_W4_VARIANT=65) vs the
# non-temporal default (63), end to end: the prefill outputs (qkv 200 MB, GLU 470 MB per 16k
# chunk) may stay in the MALL for their consumers.  Headline interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5bb; mkdir -p $O
DRTC_W4_VARIANT=65 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_gpu.py -k "w4 or mfma" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -le 1 ] || exit $rc
for r in a1 b1 a2 b2; do
  v=63; [ "${r#b}" != "$r" ] && v=65
  DRTC_W4_VARIANT=$v timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/$r.json 2> $O/$r.err || { tail -5 $O/$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$r.json'));s=d['engine_stats'];print('$r v$v', d['value'], 'decode_us', s['decode_us'], 'prefill_us', s['prefill_us'])"
done
