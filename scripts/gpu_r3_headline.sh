#!/bin/bash
# Round 3: GPU tests of the model paths touched by the hand GEMM dispatch, the headline A/B
# (hand GEMMs on prefill + decode vs the library everywhere), then a kernel-trace profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_model_real_shapes_gpu.py tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_model.log 2>&1 || { tail -30 gpurun_out/t_model.log; exit 1; }
tail -1 gpurun_out/t_model.log
timeout -k 10 400 python -u bench.py --steps ${STEPS:-10} --warmup 3 > gpurun_out/bench_hand.json 2> gpurun_out/bench_hand.err || { tail -20 gpurun_out/bench_hand.err; exit 1; }
cat gpurun_out/bench_hand.json
DRTC_W4_GEMM=0 DRTC_W4_GLU=0 timeout -k 10 400 python -u bench.py --steps ${STEPS:-10} --warmup 3 > gpurun_out/bench_lib.json 2> gpurun_out/bench_lib.err || exit 1
cat gpurun_out/bench_lib.json
if [ -n "${PROF:-}" ]; then bash scripts/gpu_prof_model.sh $PROF --steps 2 --warmup 1 > gpurun_out/prof_model.log 2>&1; echo "prof rc=$?"; fi
