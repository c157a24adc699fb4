#!/bin/bash
# rocprofv3 kernel traces (one timed step each) of the secondary BASELINE
# configurations: Gemma-2B smart reply, Mixtral context suggestions, Llama-3-70B
# Ask-AI.  Leaves gpurun_out/TAG_summary_full.md + TAG_kernel_stats.csv per config.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
prof() {  # tag, bench args...
  local tag=$1; shift
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 "$@" > "$R/gpurun_out/prof_$tag.log" 2>&1
  local rc=$?
  cd "$R"
  echo "$tag prof rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_$tag.log; return $rc; }
  local T S
  T=$(find gpurun_out/prof_$tag -name '*kernel_trace.csv' | head -1)
  S=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1)
  [ -n "$T" ] && python scripts/prof_summary.py "$T" --top 25 --full-only > gpurun_out/${tag}_summary_full.md 2>&1
  [ -n "$S" ] && cp "$S" gpurun_out/${tag}_kernel_stats.csv
  rm -rf gpurun_out/prof_$tag
  grep '"metric"' gpurun_out/prof_$tag.log | cut -c1-300
  return 0
}
prof gemma --model gemma-2b && \
prof mixtral --model mixtral-8x7b --workload suggest --batch 256 && \
prof ask70b --model llama-3-70b --workload ask --batch 256
