#!/bin/bash
# Round 6, call 2: GPU suite with the product's own exit path (no conftest join), smoke, the
# headline bench, the long-K down GEMM A/B + L2 PMC, and the current-tree
# hipGraph HIP-API trace of the headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6b; mkdir -p $O
DRTC_TEST_JOIN=0 DRTC_TEST_THREADS=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -5 $O/suite.log; echo "suite rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json | cut -c1-300
# long-K down projection: library vs gemm_w4 schedules / row groups, residual epilogue
timeout -k 10 300 python -u scripts/w4_probe.py --shape 16384,4096,14336 --epi residual --arms lib,v63:1:4,v63:1:8,v63:1:2,v63:1:16,v31:1:4,v15:1:4,v7:1:4 --iters 10 --rounds 5 > $O/down8b.log 2>&1 || { tail -20 $O/down8b.log; exit 1; }
grep -v amdgpu $O/down8b.log
timeout -k 10 300 python -u scripts/w4_probe.py --shape 16384,8192,28672 --epi residual --arms lib,v63:1:4,v63:1:8,v7:1:4 --iters 4 --rounds 4 > $O/down70b.log 2>&1 || { tail -20 $O/down70b.log; exit 1; }
grep -v amdgpu $O/down70b.log
# lm_head at the full decode batch (M = 1024): library vs gemm_w4 (persistent 256 x 256) vs gemm_xd
timeout -k 10 300 python -u scripts/w4_probe.py --shape 1024,128256,4096 --epi store --arms lib,v63:1:8,v63:1:4,v31:1:8,x1281,x281 --iters 10 --rounds 5 > $O/lmhead.log 2>&1 || { tail -20 $O/lmhead.log; exit 1; }
grep -v amdgpu $O/lmhead.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d $O/pmc_down -o pmc --output-format csv -- python3 $R/scripts/w4_probe.py --shape 16384,4096,14336 --epi residual --arms lib,v63:1:4,v63:1:8,v7:1:4 --iters 2 --rounds 1 > $O/pmc_down.log 2>&1 || { tail -5 $O/pmc_down.log; exit 1; }
cd $R
python3 scripts/pmc_summary.py $(find $O/pmc_down -name '*counter_collection.csv') > $O/pmc_down_summary.txt 2>&1; cut -c1-300 $O/pmc_down_summary.txt
rm -rf $O/pmc_down
# the decode attention's K / V addressing against the plain gather (r6c follow-up)
timeout -k 10 180 scripts/native/stream_probe > $O/stream.log 2>&1 || { tail -5 $O/stream.log; exit 1; }
grep -E "gather4k|attn_kv" $O/stream.log
# hipGraph evidence on the current tree: HIP API + kernel trace of the headline config
cd /tmp
timeout -k 10 600 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 1 --warmup 1 > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; cd $R; [ $rc -eq 0 ] || { tail -5 $O/trace.log; exit $rc; }
A=$(find $O/trace -name '*hip_api_trace.csv' | head -1); K=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python3 scripts/graph_trace_summary.py "$A" "$K" > $O/graph_trace.md && head -30 $O/graph_trace.md
python3 scripts/prof_summary.py "$K" --top 20 --full-only > $O/trace_summary_full.md
gzip -c "$K" > $O/trace_kernels.csv.gz; gzip -c "$A" > $O/trace_hip_api.csv.gz
rm -rf $O/trace
