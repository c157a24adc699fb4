#!/bin/bash
# Headline kernel trace (rocprofv3 --kernel-trace) + idle attribution per
# phase (scripts/trace_gaps.py).  Keeps the compressed trace of the run.
set -u
TAG=${1:-r2e}; shift || true
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1
rc=$?
echo "prof rc=$rc"
cd "$R"
T=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
S=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
[ -n "$T" ] && python scripts/trace_gaps.py "$T" --min-us 300 > gpurun_out/${TAG}_gaps.txt 2>&1
[ -n "$T" ] && python scripts/prof_summary.py "$T" --top 25 --full-only > gpurun_out/${TAG}_summary_full.md 2>&1
[ -n "$S" ] && cp "$S" gpurun_out/${TAG}_kernel_stats.csv
[ -n "$T" ] && gzip -c "$T" > gpurun_out/${TAG}_kernel_trace.csv.gz
rm -rf gpurun_out/prof_$TAG
cat gpurun_out/${TAG}_gaps.txt
exit $rc
