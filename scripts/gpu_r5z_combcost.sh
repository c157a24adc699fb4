#!/bin/bash
# Round 5: what the split-K combine's memory traffic costs per decode shape - the tuned split
# forms timed normally and with DRTC_XD_SLAB_TIMING=1 (zero-range slab: partial loads / stores
# dropped, protocol and instruction stream kept; results wrong, timing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5z; mkdir -p $O
P="timeout -k 10 150 python -u scripts/w4_probe.py --iters 20 --rounds 5"
run() {
  $P --shape 1024,4096,14336 --rotate 4 --arms x242,x284 &&
  $P --shape 1024,4096,4096 --rotate 12 --arms x141,x284,x242 &&
  $P --shape 256,10240,8192 --rotate 3 --arms x1243 &&
  $P --shape 256,8192,8192 --rotate 3 --arms x1244 &&
  $P --shape 256,8192,28672 --rotate 2 --arms x1244
}
{ run; } > $O/normal.log 2>&1 || { tail -20 $O/normal.log; exit 1; }
{ DRTC_XD_SLAB_TIMING=1 run; } > $O/noslab.log 2>&1 || { tail -20 $O/noslab.log; exit 1; }
paste <(grep -v amdgpu.ids $O/normal.log | python3 -c "import sys,json;[print(json.loads(l)['shape'],json.loads(l)['arm'],json.loads(l)['us_med']) for l in sys.stdin]") \
      <(grep -v amdgpu.ids $O/noslab.log | python3 -c "import sys,json;[print(json.loads(l)['us_med']) for l in sys.stdin]")
