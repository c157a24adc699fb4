#!/bin/bash
# Round 4: headline with the default 3 timed steps after 1 / 2 / 3 warmup steps, on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4aj
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in 1 2 3 1; do
  timeout -k 10 400 python -u bench.py --steps 3 --warmup $w > gpurun_out/r4aj/bench_w$w.json 2> gpurun_out/r4aj/bench_w$w.err || { tail -5 gpurun_out/r4aj/bench_w$w.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4aj/bench_w$w.json')); print($w, d['value'], d['ms_per_step'], d['engine_stats'])"
done
