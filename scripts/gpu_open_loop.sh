#!/bin/bash
# Open-loop (Poisson) smart-reply serving on one MI355X: mixed prefill+decode
# scheduling at several prompt-token budgets vs strict prefill-first, at the
# stated arrival rate; then the closed-wave headline (must not regress).
# Usage: bash scripts/gpu_open_loop.sh [rate] [requests]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
RATE=${1:-300}; N=${2:-4500}; OUT=gpurun_out/open_loop_$RATE.jsonl
: > "$OUT"
step() {  # label, args...
  local label=$1; shift
  echo "== $label $(date +%T)"
  timeout -k 10 300 python -u bench.py --warmup 1 --arrival-rate "$RATE" --requests "$N" "$@" \
    > gpurun_out/ol_$label.json 2> gpurun_out/ol_$label.err || { echo "$label failed rc=$?"; tail -20 gpurun_out/ol_$label.err; return 1; }
  cat gpurun_out/ol_$label.json >> "$OUT"; cut -c1-600 gpurun_out/ol_$label.json
}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_model_gpu.py -k "mixed or pipelined" > gpurun_out/ol_tests.log 2>&1 \
  && tail -3 gpurun_out/ol_tests.log \
  && step mixed4096 --mixed-tokens 4096 \
  && step prefill_first --no-mixed \
  && step mixed2048 --mixed-tokens 2048 \
  && step mixed8192 --mixed-tokens 8192 \
  && echo "== closed headline $(date +%T)" \
  && timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ol_headline.json 2> gpurun_out/ol_headline.err \
  && cut -c1-700 gpurun_out/ol_headline.json
