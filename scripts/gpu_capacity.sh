#!/bin/bash
# Open-loop capacity probe: Poisson arrivals above and around saturation; the
# steady_req_per_s field is the completion rate in the 30-90 % part of the
# arrival window (excludes ramp-up and the final drain).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rate in ${RATES:-350 400 450 500}; do
  timeout -k 10 300 python bench.py --warmup 1 --arrival-rate $rate --requests $((rate * 16)) \
      > gpurun_out/cap${TAG:-}_$rate.json 2> gpurun_out/cap${TAG:-}_$rate.err || { tail -5 gpurun_out/cap${TAG:-}_$rate.err; exit 1; }
  python - "$rate" "${TAG:-}" <<'PY'
import json, sys
r = json.loads(open(f"gpurun_out/cap{sys.argv[2]}_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], {k: r[k] for k in ("achieved_req_per_s", "steady_req_per_s", "steady_gen_tokens_per_s",
                                     "p50_latency_ms", "p99_latency_ms", "p50_tpot_ms", "p99_tpot_ms",
                                     "p50_ttft_ms")}, r["engine_stats"].get("mixed_steps"))
PY
done
