#!/bin/bash
# Round 5: decode attention at the headline shape (B 1024, ctx 150-200) against the chip's plain
# read bandwidth on the same box (a 4 GiB bf16 sum and copy).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5ai; mkdir -p $O
timeout -k 10 300 python -u scripts/decode_attn_bench.py 3 llama8b > $O/attn.log 2>&1 || { tail -20 $O/attn.log; exit 1; }
grep -v amdgpu $O/attn.log | head -12
timeout -k 10 120 python -u - > $O/bw.log 2>&1 <<'PY' || { tail -5 $O/bw.log; exit 1; }
import torch
x = torch.randn(2 << 30, device="cuda", dtype=torch.bfloat16)  # 4 GiB
y = torch.empty_like(x)
def t(fn, it=10):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / it
ms = t(lambda: x.sum(dtype=torch.float32))
print(f"read (sum) {x.numel() * 2 / ms / 1e9:.2f} TB/s")
ms = t(lambda: y.copy_(x))
print(f"copy {2 * x.numel() * 2 / ms / 1e9:.2f} TB/s (read + write)")
PY
cat $O/bw.log
