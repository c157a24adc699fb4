#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_full_suite.sh || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_r3d.json 2> gpurun_out/bench_r3d.err || { tail -20 gpurun_out/bench_r3d.err; exit 1; }
cat gpurun_out/bench_r3d.json
