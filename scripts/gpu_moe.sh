#!/bin/bash
# MoE kernel validation + Mixtral bench/profile on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -k "moe or mixtral" > gpurun_out/pytest_moe.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_moe.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/moe_bench.py > gpurun_out/moe_bench.log 2>&1
rc=$?; cat gpurun_out/moe_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --model mixtral-8x7b --workload suggest --batch 256 --steps 2 --warmup 1 > gpurun_out/bench_mix.json 2> gpurun_out/bench_mix.err
rc=$?; tail -3 gpurun_out/bench_mix.err; cat gpurun_out/bench_mix.json; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_mix" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --model mixtral-8x7b --workload suggest --batch 256 --steps 1 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_mix.log" 2>&1
echo "prof rc=$?"
