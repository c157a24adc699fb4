#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -k "moe or mixtral" > gpurun_out/pytest_moe.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_moe.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python scripts/moe_bench.py > gpurun_out/moe_bench2.log 2>&1
rc=$?; cat gpurun_out/moe_bench2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --model mixtral-8x7b --workload suggest --batch 256 --steps 2 --warmup 1 > gpurun_out/bench_mix2.json 2> gpurun_out/bench_mix2.err
rc=$?; tail -2 gpurun_out/bench_mix2.err; cut -c1-400 gpurun_out/bench_mix2.json; exit $rc
