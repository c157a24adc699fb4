#!/bin/bash
# Round 5: xd tests on the final combine build, re-tune gemm_xd for Llama-3-70B (TP1 decode
# buckets up to 256, TP8 shard shapes) with the batched combine, merge, then the 70B ask-AI wave
# at batch 256 and the headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5w; mkdir -p $O
( while true; do date >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_gpu.py tests/test_kernels_gpu.py -k "xd or splitk or moe" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python -u scripts/tune_xd.py --configs llama-3-70b:1,llama-3-70b:8 \
  --ms 128,160,192,224,256,320,384,448,512,640,768,896,1024 --out $O/xd_tuned.json 2>&1 | grep -v amdgpu.ids > $O/tune.log || exit 1
tail -1 $O/tune.log
python scripts/tune_gemms.py --merge $O/xd_tuned.json || exit 1
cp distributed-real-time-chat-and-collaboration-tool_amd/ops/tuned/gemm_gfx950.json $O/
timeout -k 10 600 python -u bench.py --model llama-3-70b --workload ask --batch 256 --steps 3 --warmup 1 \
  > $O/b70_256.json 2> $O/b70_256.err || { tail -5 $O/b70_256.err; exit 1; }
cut -c1-400 $O/b70_256.json
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
echo "engine $(python3 -c "import json;print(json.load(open('$O/engine.json'))['value'])")"
