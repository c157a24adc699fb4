#!/bin/bash
# Throughput knee of the secondary models at larger engine batches (deadline check in the
# JSON's p50): Mixtral suggestions at 768 / 1024, Gemma-2B smart reply at 2048.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local tag=$1; shift
  DRTC_TIME_DECODE=1 timeout -k 10 400 python bench.py "$@" > gpurun_out/knee_$tag.json 2> gpurun_out/knee_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/knee_$tag.err; exit 1; }
  python - gpurun_out/knee_$tag.json "$tag" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], d["config"]["global_batch"], d["value"], "tok/s  p50", d["p50_latency_ms"], "p99", d["p99_latency_ms"], "ms")
PY
  grep "decode graph" gpurun_out/knee_$tag.err
}
run mix768 --model mixtral-8x7b --workload suggest --batch 768 --steps 2 && \
run mix1024 --model mixtral-8x7b --workload suggest --batch 1024 --steps 2 && \
run mix512 --model mixtral-8x7b --workload suggest --batch 512 --steps 2 && \
run gemma2048 --model gemma-2b --batch 2048 --steps 3 && \
run gemma1024 --model gemma-2b --batch 1024 --steps 3 && \
run smart1024 --steps 3
[ "${BAL_AB:-0}" = "1" ] && DRTC_PREFILL_BALANCE=0 run smart_bal0 --steps 4 && run smart_bal1 --steps 4 && \
  DRTC_PREFILL_BALANCE=0 run smart_bal0b --steps 4 && run smart_bal1b --steps 4
