#!/bin/bash
# Round 5 baseline on this round's first box: smoke, headline bench, prefill GEMM probe
# (gemm_w4 v63 vs hipBLASLt on the four Llama-3-8B prefill shapes, interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 10 --rounds 5"
{
$P --shape 16384,6144,4096 --arms lib,v63 --group-m 4 &&
$P --shape 16384,4096,4096 --epi residual --arms lib,v63 --group-m 4 &&
$P --shape 16384,28672,4096 --epi silu --arms lib,v63 &&
$P --shape 16384,4096,14336 --arms lib,v63 --group-m 2
} > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | cut -c1-200
