#!/bin/bash
# Round 3: sampler with two 1024-thread workgroups per CU (DRTC_SAMPLER_OCC=2: <= 64 VGPRs,
# 2-deep load unroll) against one per CU - sampler tests under both, kernel bench, headline A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3v
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
for o in 2 1; do
  DRTC_SAMPLER_OCC=$o timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_kernels_gpu.py -k sample > gpurun_out/r3v/tests_occ$o.log 2>&1 || { tail -20 gpurun_out/r3v/tests_occ$o.log; exit 1; }
  tail -1 gpurun_out/r3v/tests_occ$o.log
  DRTC_SAMPLER_OCC=$o timeout -k 10 200 python -u scripts/sampler_bench.py > gpurun_out/r3v/bench_occ$o.log 2>&1 || exit 1
done
paste -d'\n' gpurun_out/r3v/bench_occ1.log gpurun_out/r3v/bench_occ2.log | cut -c1-160
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3v/ab_$tag.json 2> gpurun_out/r3v/ab_$tag.err || { tail -5 gpurun_out/r3v/ab_$tag.err; return 1; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/r3v/ab_$tag.json'));print(d['value'],d['ms_per_step'])")"; }
run occ2 DRTC_SAMPLER_OCC=2 && run occ1 DRTC_SAMPLER_OCC=1 && run occ2b DRTC_SAMPLER_OCC=2 && run occ1b DRTC_SAMPLER_OCC=1
