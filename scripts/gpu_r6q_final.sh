#!/bin/bash
# Round 6, final tree: GPU suite (product exit path only), smoke, the current-tree hipGraph
# HIP-API + kernel trace of the headline, and the Llama-3-70B ask rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6q; mkdir -p $O
DRTC_TEST_THREADS=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; echo "suite rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 1 --warmup 1 > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; cd $R; [ $rc -eq 0 ] || { tail -5 $O/trace.log; exit $rc; }
A=$(find $O/trace -name '*hip_api_trace.csv' | head -1); K=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python3 scripts/graph_trace_summary.py "$A" "$K" > $O/graph_trace.md && grep -iE "graph|kernels per" $O/graph_trace.md | head -12
python3 scripts/prof_summary.py "$K" --top 20 --full-only > $O/trace_summary_full.md
gzip -c "$K" > $O/trace_kernels.csv.gz; gzip -c "$A" > $O/trace_hip_api.csv.gz
rm -rf $O/trace
bash scripts/gpu_r6h_configs.sh r6q l70_256a "--model llama-3-70b --workload ask --batch 256 --steps 2 --warmup 1" \
  l70_256b "--model llama-3-70b --workload ask --batch 256 --steps 2 --warmup 1" \
  l70_224 "--model llama-3-70b --workload ask --batch 224 --steps 2 --warmup 1" || exit 1
