#!/bin/bash
# Round 5: the split-K combine now batches its slab loads (profiles/r5u): headline on the old
# table, re-tune gemm_xd for Llama-3-8B and Gemma-2B at every decode bucket, merge, headline
# again on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5v; mkdir -p $O
( while true; do date >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine_old.json 2> $O/engine_old.err || { tail -5 $O/engine_old.err; exit 1; }
echo "engine old table $(python3 -c "import json;print(json.load(open('$O/engine_old.json'))['value'])")"
timeout -k 10 900 python -u scripts/tune_xd.py --configs llama-3-8b:1,gemma-2b:1 \
  --out $O/xd_tuned.json 2>&1 | grep -v amdgpu.ids > $O/tune.log || exit 1
tail -1 $O/tune.log
python scripts/tune_gemms.py --merge $O/xd_tuned.json || exit 1
cp distributed-real-time-chat-and-collaboration-tool_amd/ops/tuned/gemm_gfx950.json $O/
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine_new.json 2> $O/engine_new.err || { tail -5 $O/engine_new.err; exit 1; }
echo "engine new table $(python3 -c "import json;print(json.load(open('$O/engine_new.json'))['value'])")"
