#!/bin/bash
# Kernel trace of an open-loop run (mixed steps) + GPU idle accounting.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
RATE=${1:-400}; N=${2:-3000}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_ol" -o run -- python3 "$R/bench.py" --warmup 1 --arrival-rate "$RATE" --requests "$N" > "$R/gpurun_out/prof_ol.log" 2>&1
rc=$?
cd "$R"
T=$(find gpurun_out/prof_ol -name '*kernel_trace.csv' | head -1)
[ -n "$T" ] && python - "$T" <<'PY' > gpurun_out/ol_idle.txt
import csv, sys
rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:160]))
rows.sort()
# the open-loop window: last 60 % of the trace (after warm-up / graph capture)
t0 = rows[int(len(rows) * 0.4)][0]
rows = [r for r in rows if r[0] >= t0]
span = (rows[-1][1] - rows[0][0]) / 1e6
busy = sum(b - a for a, b, _ in rows) / 1e6
gaps = sorted(((b[0] - a[1]) / 1e3, a[2], b[2]) for a, b in zip(rows, rows[1:]))
big = [g for g in gaps if g[0] > 100]
print(f"window {span:.1f} ms, kernel-busy {busy:.1f} ms ({100 * busy / span:.1f} %), {len(rows)} kernels")
print(f"gaps > 100 us: {len(big)}, total {sum(g[0] for g in big) / 1e3:.1f} ms")
agg = {}
for g, a, b in big:
    k = f"{a} -> {b}"
    agg[k] = agg.get(k, 0) + g
for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:10]:
    print(f"  {v / 1e3:8.1f} ms  {k}")
# kernel-time breakdown of the window by kernel (GEMMs grouped by macro tile)
import re
tot = {}
cnt = {}
for a, b, n in rows:
    m = re.search(r"MT\d+x\d+x\d+", n)
    k = ("GEMM " + m.group(0)) if m else n
    tot[k] = tot.get(k, 0) + (b - a)
    cnt[k] = cnt.get(k, 0) + 1
print("kernel time in the window:")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
    print(f"  {v / 1e6:8.1f} ms {100 * v / 1e6 / busy:5.1f} %  {cnt[k]:6d}x  {k}")
PY
cat gpurun_out/ol_idle.txt; tail -2 gpurun_out/prof_ol.log | cut -c1-400
rm -rf gpurun_out/prof_ol
exit $rc
