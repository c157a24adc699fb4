#!/bin/bash
# Kernel-trace profiles of the headline with the hand GEMMs and with the library everywhere,
# on the same box (per-kernel in-situ comparison).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_prof_model.sh r3c_hand --steps 2 --warmup 1 > gpurun_out/prof_hand.log 2>&1 || exit 1
DRTC_W4_GEMM=0 DRTC_W4_GLU=0 bash scripts/gpu_prof_model.sh r3c_lib --steps 2 --warmup 1 > gpurun_out/prof_lib.log 2>&1 || exit 1
echo ok
