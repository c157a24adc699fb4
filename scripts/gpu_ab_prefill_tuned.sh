#!/bin/bash
# A/B of the prefill-sized tuned GEMM entries on the headline bench (alternating runs, one box).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
for i in 1 2; do
  for on in 1 0; do
    DRTC_PREFILL_TUNED=$on timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
        > gpurun_out/ab_prefill_${on}_$i.json 2> gpurun_out/ab_prefill_${on}_$i.log || exit $?
    echo "on=$on run=$i $(python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['p50_ttft_ms'])" gpurun_out/ab_prefill_${on}_$i.json)"
  done
done
