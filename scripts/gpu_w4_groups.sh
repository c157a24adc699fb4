#!/bin/bash
# Row-group size of the XCD-aware tile order (gemm_w4) per prefill shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
: > gpurun_out/probe_groups.log
for spec in "16384,28672,4096 silu 4 8 16 32" "16384,4096,4096 residual 2 4 8 16" "16384,6144,4096 store 2 4 8 16" "16384,4096,14336 residual 1 2 3"; do
  set -- $spec
  shape=$1; epi=$2; shift 2
  for gm in "$@"; do
    timeout -k 10 200 python -u scripts/w4_probe.py --shape $shape --epi $epi --arms ${ARMS:-v13} --group-m $gm --rounds 5 | sed "s/}/, \"gm\": $gm}/" >> gpurun_out/probe_groups.log 2>&1 || exit 1
  done
done
grep -v amdgpu gpurun_out/probe_groups.log
