#!/usr/bin/env python3
"""GPU-idle accounting of the timed step in a rocprofv3 kernel trace of bench.py.

The timed step is everything after the last host gap longer than --gap-ms
(prompt building between warm-up and timing).  Prints the step's kernel span,
the summed kernel-busy time, where prefill ends / decode starts, and every
idle gap longer than --min-us inside the step.

usage: trace_gaps.py gpurun_out/TAG_kernel_trace.csv.gz [--gap-ms 20] [--min-us 500]
"""
import csv
import gzip
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def main():
    path = sys.argv[1]
    gap_ms = float(sys.argv[sys.argv.index("--gap-ms") + 1]) if "--gap-ms" in sys.argv else 20.0
    min_us = float(sys.argv[sys.argv.index("--min-us") + 1]) if "--min-us" in sys.argv else 500.0
    opener = gzip.open if path.endswith(".gz") else open
    rows = []
    with opener(path, "rt") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    cut = [i for i, (a, b) in enumerate(zip(rows, rows[1:])) if b[0] - a[1] > gap_ms * 1e6]
    st = rows[cut[-1] + 1:] if cut else rows
    s0 = st[0][0]
    span = (st[-1][1] - s0) / 1e6
    busy = sum(b - a for a, b, _ in st) / 1e6
    print(f"timed step: span {span:.1f} ms, kernel-busy {busy:.1f} ms ({100 * busy / span:.1f} %), "
          f"{len(st)} kernels")
    dec = [r for r in st if r[2].startswith("drtc::paged_decode")]
    if dec:
        print(f"first decode attention at {(dec[0][0] - s0) / 1e6:.1f} ms (prefill phase before it)")
    for a, b in zip(st, st[1:]):
        g = (b[0] - a[1]) / 1e3
        if g > min_us:
            print(f"idle {g:.0f} us at {(a[1] - s0) / 1e6:.1f} ms: {a[2]} -> {b[2]}")
    # idle attribution: summed gap per (previous kernel -> next kernel), split
    # into the prefill phase (before the first decode attention) and decode
    t_dec = dec[0][0] if dec else st[-1][1] + 1
    for phase, sel in (("prefill", lambda t: t < t_dec), ("decode", lambda t: t >= t_dec)):
        agg, n_gap, tot = {}, {}, 0.0
        for a, b in zip(st, st[1:]):
            if not sel(b[0]):
                continue
            g = max(0, b[0] - a[1]) / 1e3
            k = f"{a[2]} -> {b[2]}"
            agg[k] = agg.get(k, 0.0) + g
            n_gap[k] = n_gap.get(k, 0) + 1
            tot += g
        print(f"\n{phase}: idle between kernels {tot / 1e3:.1f} ms; top transitions:")
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:12]:
            print(f"  {v / 1e3:8.2f} ms  {n_gap[k]:6d} x  mean {v / n_gap[k]:7.1f} us  {k}")


if __name__ == "__main__":
    main()
