#!/bin/bash
# Secondary configs at batch sizes chosen against the reference's per-feature deadlines
# (summarize 10 s node->LLM, ask-AI 10 s, suggestions 20 s: ref server/raft_node.py:2084,2126,2187).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # tag, bench args... (env prefixes pass through)
  local tag=$1; shift
  DRTC_TIME_DECODE=1 timeout -k 10 400 python bench.py "$@" > gpurun_out/dl_$tag.json 2> gpurun_out/dl_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/dl_$tag.err; exit 1; }
  echo "$tag $(cut -c1-160 gpurun_out/dl_$tag.json)"; python - gpurun_out/dl_$tag.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("   ", d["config"]["global_batch"], d["value"], "tok/s  p50", d["p50_latency_ms"], "p99", d["p99_latency_ms"], "ms")
PY
}
run sum1024 --workload summarize --batch 1024 --steps 2 && \
run sum768 --workload summarize --batch 768 --steps 2 && \
run mix512 --model mixtral-8x7b --workload suggest --batch 512 --steps 2 && \
run ask128 --model llama-3-70b --workload ask --batch 128 --steps 1 && \
run ask192 --model llama-3-70b --workload ask --batch 192 --steps 1
[ "${GC_AB:-0}" = "1" ] && run h_gc1 --steps 5 --warmup 2 && \
  DRTC_GC_FREEZE=0 run h_gc0 --steps 5 --warmup 2 && run h_gc1b --steps 5 --warmup 2 && \
  DRTC_GC_FREEZE=0 run h_gc0b --steps 5 --warmup 2
