#!/bin/bash
# Round 5: MoE router logits on the transposed skinny HIP GEMM (no library GEMM in the MoE
# layer): router / EP / MoE fp32 tests, the Mixtral suggestions wave at batch 1024, and a
# kernel trace of one Mixtral step (which library kernels remain).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5ae; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_expert_parallel_gpu.py -k "router or moe or ep_" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --workload suggest --batch 1024 --steps 3 --warmup 1 \
  > $O/mixtral1024.json 2> $O/mixtral1024.err || { tail -5 $O/mixtral1024.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/mixtral1024.json'));print('mixtral', d['value'], d.get('p50_latency_ms'))"
bash scripts/gpu_prof_model.sh r5ae_mix --model mixtral-8x7b --workload suggest --batch 1024 --steps 1 --warmup 1 > $O/prof.out 2>&1
rc=$?; tail -2 $O/prof.out; [ $rc -eq 0 ] || exit $rc
mv gpurun_out/r5ae_mix* $O/ 2>/dev/null
grep -i "hipblaslt\|Cijk" $O/r5ae_mix_summary_full.md | head -10
