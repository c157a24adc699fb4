#!/bin/bash
# Round 6: balanced decode attention item order - slots sorted by context length (engine) +
# every odd round of the persistent kernel's item deal mirrored - numerics, kernel A/B on
# random vs sorted contexts, headline A/B (DRTC_SORT_SLOTS=0: unsorted slots).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_decode_micro_gpu.py tests/test_model_gpu.py tests/test_model_real_shapes_gpu.py -k "decode or paged or rope or micro or serving or engine or graph or mixed" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/decode_attn_cap.py 0 random,sorted > $O/attn.log 2>&1 || { tail -5 $O/attn.log; exit 1; }
grep -v amdgpu $O/attn.log
for i in 1 2; do
  for so in 256 0; do
    DRTC_SORT_SLOTS=$so DRTC_TIME_DECODE=1 timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 > $O/bench_s${so}_$i.json 2> $O/bench_s${so}_$i.err || { tail -20 $O/bench_s${so}_$i.err; exit 1; }
    echo "bench sort_min=$so run $i: $(python -c "import json;d=json.load(open('$O/bench_s${so}_$i.json'));print(d['value'],d['p50_latency_ms'])") $(grep 'decode graph' $O/bench_s${so}_$i.err)"
  done
done
