#!/bin/bash
# Round 6, shipped tree: GPU suite + smoke, the headline bench twice, and rocprofv3 kernel
# anatomies of the Mixtral and Llama-3-70B configurations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6ad; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -2 $O/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
cut -c1-200 $O/bench_default.json
bash scripts/gpu_r6h_configs.sh r6ad l8_1024a "--steps 6 --warmup 2" l8_1024b "--steps 6 --warmup 2" || exit 1
bash scripts/gpu_prof_model.sh r6ad_mix --model mixtral-8x7b --workload suggest --batch 1024 --steps 2 --warmup 1 || exit 1
head -30 gpurun_out/r6ad_mix_summary.md
bash scripts/gpu_prof_model.sh r6ad_l70 --model llama-3-70b --workload ask --batch 256 --steps 1 --warmup 1 || exit 1
head -30 gpurun_out/r6ad_l70_summary.md
