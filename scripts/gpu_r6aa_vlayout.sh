#!/bin/bash
# Round 6: V-cache slot-row layout ([4][D][8], one 16-B P.V operand load per fragment) - the
# GPU suite, decode attention timing, headline and Mixtral / 70B rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6aa; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u scripts/decode_attn_cap.py 0 random,sorted > $O/attn.log 2>&1 || { tail -5 $O/attn.log; exit 1; }
grep '"B"' $O/attn.log
bash scripts/gpu_r6h_configs.sh r6aa l8_1024a "--steps 6 --warmup 2" l8_1024b "--steps 6 --warmup 2" \
  l8_512 "--batch 512 --steps 4 --warmup 1" \
  mix_1024 "--model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1" \
  l70_256 "--model llama-3-70b --workload ask --batch 256 --steps 2 --warmup 1" || exit 1
