#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
run() { name=$1; shift; timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err; rc=$?; echo "bench $name rc=$rc"; cut -c1-330 gpurun_out/bench_$name.json; [ $rc -eq 0 ] || exit $rc; }
run default
run gemma_smart --model gemma-2b --batch 1024
run llama8b_summarize --workload summarize --batch 512
run mixtral_suggest --model mixtral-8x7b --workload suggest --batch 256
run llama70b_ask --model llama-3-70b --workload ask --batch 256
