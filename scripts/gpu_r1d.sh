#!/bin/bash
# Round-1 "d" measurements: default bench (+ rocprofv3 kernel trace) and the
# service-level load driver on Llama-3-8B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
true
true
timeout -k 10 600 python scripts/service_bench.py --model llama-3-8b --mode direct --requests 2048 --concurrency 1024 --max-batch 1024 > gpurun_out/service_direct.json 2> gpurun_out/service_direct.err
rc=$?; tail -2 gpurun_out/service_direct.err; cut -c1-700 gpurun_out/service_direct.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python scripts/service_bench.py --model llama-3-8b --mode raft --requests 1024 --concurrency 512 --max-batch 1024 > gpurun_out/service_raft.json 2> gpurun_out/service_raft.err
rc=$?; tail -2 gpurun_out/service_raft.err; cut -c1-700 gpurun_out/service_raft.json; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_d" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_d.log" 2>&1
echo "prof rc=$?"
