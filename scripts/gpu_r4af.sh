#!/bin/bash
# Round 4: the in-tree table with the non-temporal gemm_xd tuning: router / gemm tests, the
# Llama-3-70B ask wave at batch 256 / 224 and its kernel-trace anatomy at 256.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4af
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py > gpurun_out/r4af/tests.log 2>&1 || { tail -30 gpurun_out/r4af/tests.log; exit 1; }
tail -1 gpurun_out/r4af/tests.log
for b in 256 224; do
  timeout -k 10 600 python -u bench.py --model llama-3-70b --workload ask --batch $b --steps 3 --warmup 1 \
    > gpurun_out/r4af/b70_$b.json 2> gpurun_out/r4af/b70_$b.err || { tail -5 gpurun_out/r4af/b70_$b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4af/b70_$b.json')); print($b, d['value'], d['p50_latency_ms'], d['p50_ttft_ms'])"
done
bash scripts/gpu_prof_model.sh r4af_70b --model llama-3-70b --workload ask --batch 256 --steps 1 --warmup 1 > gpurun_out/r4af/prof.out 2>&1
rc=$?; tail -3 gpurun_out/r4af/prof.out; [ $rc -eq 0 ] || exit $rc
grep -A 12 '^\*\*decode' gpurun_out/r4af_70b_summary.md
