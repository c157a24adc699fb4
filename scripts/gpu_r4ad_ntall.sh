#!/bin/bash
# Round 4: re-tune gemm_xd at the Llama-3-8B full-batch buckets with the non-temporal forms
# among the candidates at every M, merge, then the headline A/B (re-tuned table vs the
# committed one) on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4ad
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
T=distributed-real-time-chat-and-collaboration-tool_amd/ops/tuned/gemm_gfx950.json
cp $T gpurun_out/r4ad/table_before.json
timeout -k 10 600 python -u scripts/tune_xd.py --configs llama-3-8b:1 --ms 768,896,1024 --nt-any \
  --out gpurun_out/r4ad/xd_tuned.json 2>&1 | grep -v amdgpu.ids > gpurun_out/r4ad/tune.log || exit 1
tail -1 gpurun_out/r4ad/tune.log
python scripts/tune_gemms.py --merge gpurun_out/r4ad/xd_tuned.json || exit 1
cp $T gpurun_out/r4ad/table_after.json
b() {  # tag
  timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4ad/bench_$1.json 2> gpurun_out/r4ad/bench_$1.err || { tail -5 gpurun_out/r4ad/bench_$1.err; return 1; }
  echo $1 $(cut -c1-140 gpurun_out/r4ad/bench_$1.json)
}
b after && cp gpurun_out/r4ad/table_before.json $T && b before && cp gpurun_out/r4ad/table_after.json $T && b after2
