#!/bin/bash
# Round 5: per-CU LDS-DMA ingest without MFMA on the decode-GEMM access pattern
# (scripts/native/ingest_probe.hip), and gemm_ring (3 K stages in flight) on the decode
# gate_up + GLU at the headline batch against gemm_w4 (1 K tile in flight).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 120 ./scripts/native/ingest_probe > $O/ingest.log 2>&1 || { tail -20 $O/ingest.log; exit 1; }
cat $O/ingest.log
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
$P --shape 1024,28672,4096 --epi silu --rotate 3 --arms v63,r4,r8 --group-m 4 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | cut -c1-200
