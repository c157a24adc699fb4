#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV of bench.py by engine phase.

Each forward pass ends with the fused sampler kernel; the kernels since the
previous sampler form one pass, classified as prefill (it contains the
prefill attention kernel) or decode (paged decode attention).  Prints, per
phase: passes, mean GPU wall per pass, mean busy time per pass, and the
per-kernel breakdown (shortened names) - a markdown table for profiles/.

usage: prof_summary.py run_kernel_trace.csv [--top 15] [--full-only]

--full-only keeps, per phase, only the passes whose kernel-busy time is at
least 80 % of the phase's largest pass (drops the graph-capture warm-up
passes of the small batch buckets, so decode rows describe the full batch).
"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    if name.startswith("Cijk") or name.startswith("Custom_Cijk"):
        m = re.search(r"MT(\d+x\d+x\d+)", name)
        return f"hipBLASLt GEMM MT{m.group(1) if m else '?'}"
    m = re.search(r"drtc::(\w+)", name) or re.search(r"drtc(\d+)(\w+?)E", name)
    if "drtc" in name:
        for k in ("paged_decode_persist_kernel", "paged_decode_wave_kernel", "paged_decode_kernel",
                  "decode_reduce_kernel", "prefill_attn_persist_kernel", "prefill_attn_kernel",
                  "kv_write_v_kernel", "midm_reduce_kernel", "midm_kernel", "gemm_dec_kernel",
                  "gemm_w4_kernel", "gemm256", "skinny", "rmsnorm_kernel", "act_glu_kernel", "rope_kv_kernel",
                  "sample_kernel", "moe_", "allreduce"):
            if k in name:
                return "drtc::" + k
    if "at::native" in name:
        m = re.search(r"at::native::(?:\(anonymous namespace\)::)?(\w+)", name)
        return "torch::" + (m.group(1) if m else "kernel")
    return name[:60]


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 15
    rows = []
    opener = __import__("gzip").open if path.endswith(".gz") else open
    with opener(path, "rt") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    passes = []
    cur = []
    for r in rows:
        cur.append(r)
        if r[2] == "drtc::sample_kernel":
            passes.append(cur)
            cur = []
    full_only = "--full-only" in sys.argv
    phase_k = {"prefill": collections.Counter(), "decode": collections.Counter()}
    phase_n = collections.Counter()
    phase_wall = collections.Counter()
    phase_busy = collections.Counter()
    phase_cnt = collections.Counter()
    def phase_of(p):
        names = {x[2] for x in p}
        if any("distribution_" in n for n in names):
            return None  # random weight init before the first forward
        return ("prefill" if any(n.startswith("drtc::prefill_attn") for n in names) else
                "decode" if any(n.startswith("drtc::paged_decode") for n in names) else None)

    busy_max = collections.Counter()
    for p in passes:
        ph = phase_of(p)
        if ph:
            busy_max[ph] = max(busy_max[ph], sum(e - s for s, e, _ in p))
    for p in passes:
        ph = phase_of(p)
        if ph is None:
            continue
        if full_only and sum(e - s for s, e, _ in p) < 0.8 * busy_max[ph]:
            continue
        # drop leading non-forward kernels (copies etc. are not kernels here)
        phase_n[ph] += 1
        phase_cnt[ph] += len(p)
        phase_wall[ph] += p[-1][1] - p[0][0]
        for s, e, n in p:
            phase_k[ph][n] += e - s
            phase_busy[ph] += e - s
    if "--gaps" in sys.argv:
        # where a pass's wall goes beyond its kernels: idle gaps inside the pass by the
        # (previous kernel -> next kernel) transition, and the gap BEFORE each pass's first
        # kernel (host work between passes, not inside the wall)
        for ph in ("prefill", "decode"):
            agg, cnt = collections.Counter(), collections.Counter()
            n = 0
            for p in passes:
                if phase_of(p) != ph or (full_only and sum(e - s for s, e, _ in p) < 0.8 * busy_max[ph]):
                    continue
                n += 1
                end = p[0][1]
                for (s0, e0, n0), (s1, e1, n1) in zip(p, p[1:]):
                    end = max(end, e0)
                    if s1 > end:
                        agg[f"{n0} -> {n1}"] += s1 - end
                        cnt[f"{n0} -> {n1}"] += 1
            if n:
                print(f"\n{ph}: idle inside a pass {sum(agg.values()) / n / 1e6:.3f} ms / pass; top:")
                for k, v in agg.most_common(8):
                    print(f"  {v / n / 1e6:8.3f} ms/pass  {cnt[k] / n:6.1f} x/pass  {k}")
        print()
    print("| phase | passes | mean GPU wall / pass (ms) | mean kernel-busy / pass (ms) | kernels / pass |")
    print("|---|---|---|---|---|")
    for ph in ("prefill", "decode"):
        if phase_n[ph]:
            print(f"| {ph} | {phase_n[ph]} | {phase_wall[ph] / phase_n[ph] / 1e6:.3f} | "
                  f"{phase_busy[ph] / phase_n[ph] / 1e6:.3f} | {phase_cnt[ph] / phase_n[ph]:.0f} |")
    for ph in ("prefill", "decode"):
        if not phase_n[ph]:
            continue
        tot = sum(phase_k[ph].values())
        print(f"\n**{ph}** (per pass)\n\n| kernel | ms / pass | share |\n|---|---|---|")
        for n, t in phase_k[ph].most_common(top):
            print(f"| {n} | {t / phase_n[ph] / 1e6:.3f} | {100 * t / tot:.1f}% |")


if __name__ == "__main__":
    main()
