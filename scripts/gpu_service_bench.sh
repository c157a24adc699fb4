#!/bin/bash
# Service-level load driver on Llama-3-8B: gRPC clients -> llm.LLMService
# directly, and through the Raft leader (raft.RaftNode/GetSmartReply).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python scripts/service_bench.py --model llama-3-8b --mode direct --requests 2048 --concurrency 1024 --max-batch 1024 > gpurun_out/service_direct.json 2> gpurun_out/service_direct.err
rc=$?; tail -2 gpurun_out/service_direct.err; cut -c1-700 gpurun_out/service_direct.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python scripts/service_bench.py --model llama-3-8b --mode raft --requests 1024 --concurrency 512 --max-batch 1024 > gpurun_out/service_raft.json 2> gpurun_out/service_raft.err
rc=$?; tail -2 gpurun_out/service_raft.err; cut -c1-700 gpurun_out/service_raft.json; [ $rc -ne 0 ] && exit $rc
