#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_pmc_w4.sh qkv2 --shape 16384,6144,4096 --epi store --arms lib,v7 --group-m 4 > gpurun_out/pmc_w4.log 2>&1 || { tail gpurun_out/pmc_w4.log; exit 1; }
bash scripts/gpu_pmc_w4.sh down2 --shape 16384,4096,14336 --epi residual --arms lib,v7 --group-m 2 >> gpurun_out/pmc_w4.log 2>&1 || exit 1
echo ok
