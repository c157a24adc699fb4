#!/bin/bash
# Timed bench + rocprofv3 kernel trace of one bench.py configuration.
# usage: gpu_prof_model.sh TAG [bench.py args...]
# Leaves gpurun_out/TAG.json (timed run), TAG_summary.md (per-phase kernel
# breakdown) and TAG_kernel_stats.csv; the raw trace is deleted (size cap).
set -u
TAG=$1; shift
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
DRTC_TIME_DECODE=1 timeout -k 10 400 python bench.py "$@" > gpurun_out/$TAG.json 2> gpurun_out/$TAG.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1
rc=$?
echo "prof rc=$rc"
cd "$R"
T=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
S=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
[ -n "$T" ] && python scripts/prof_summary.py "$T" --top 20 > gpurun_out/${TAG}_summary.md && python scripts/prof_summary.py "$T" --top 25 --full-only > gpurun_out/${TAG}_summary_full.md
[ -n "$S" ] && cp "$S" gpurun_out/${TAG}_kernel_stats.csv
[ -n "$T" ] && gzip -c "$T" > gpurun_out/${TAG}_kernel_trace.csv.gz
rm -rf gpurun_out/prof_$TAG
exit $rc
