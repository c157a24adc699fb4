#!/bin/bash
# Timed bench.py run of every BASELINE configuration that fits one GPU.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # tag, bench args...
  local tag=$1; shift
  DRTC_TIME_DECODE=1 timeout -k 10 400 python bench.py "$@" > gpurun_out/cfg_$tag.json 2> gpurun_out/cfg_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/cfg_$tag.err; exit 1; }
  echo "$tag $(cut -c1-220 gpurun_out/cfg_$tag.json)"
}
run smart8b
run gemma --model gemma-2b
run summarize8b --workload summarize --batch 512
run mixtral --model mixtral-8x7b --workload suggest --batch 256
run ask70b --model llama-3-70b --workload ask --batch 256 --steps 1
