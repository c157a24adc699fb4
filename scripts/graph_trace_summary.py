#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--hip-trace --kernel-trace`` run of bench.py: which HIP API calls
enqueued the kernels, and how many kernels each ``hipGraphLaunch`` replayed.

Kernels carry the correlation id of the API call that enqueued them, so the kernels of one
graph replay share the id of its ``hipGraphLaunch``.  Prints (markdown): the API-call table,
the kernels-per-hipGraphLaunch histogram with the per-launch GPU span, and the kernel names of
the most common replay (one decode step).

usage: graph_trace_summary.py <hip_api_trace.csv> <kernel_trace.csv>
"""
import collections
import csv
import sys


def rows(path):
    with open(path, newline="") as f:
        yield from csv.DictReader(f)


def main():
    api_path, ker_path = sys.argv[1], sys.argv[2]
    api = {}
    calls = collections.Counter()
    dur = collections.Counter()
    for r in rows(api_path):
        fn = r.get("Function") or r.get("Operation") or "?"
        cid = r.get("Correlation_Id")
        api[cid] = fn
        calls[fn] += 1
        try:
            dur[fn] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        except (KeyError, ValueError):
            pass
    by_cid = collections.defaultdict(list)
    for r in rows(ker_path):
        by_cid[r.get("Correlation_Id")].append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "?")))
    launched_by = collections.Counter()
    for cid, ks in by_cid.items():
        launched_by[api.get(cid, "(no API record)")] += len(ks)
    print("| HIP API call | calls | host ms (traced) | kernels it enqueued |")
    print("|---|---|---|---|")
    for fn, n in calls.most_common(14):
        print(f"| {fn} | {n} | {dur[fn]:.1f} | {launched_by.get(fn, 0)} |")
    graph = [(cid, ks) for cid, ks in by_cid.items() if api.get(cid) == "hipGraphLaunch"]
    hist = collections.Counter(len(ks) for _, ks in graph)
    print(f"\n{len(graph)} hipGraphLaunch calls replayed kernels; kernels per launch:\n")
    print("| kernels per hipGraphLaunch | launches | median GPU span per launch (ms) |")
    print("|---|---|---|")
    for nk, n in sorted(hist.items(), key=lambda t: -t[1]):
        spans = sorted((max(e for _, e, _ in ks) - min(s for s, _, _ in ks)) / 1e6
                       for _, ks in graph if len(ks) == nk)
        print(f"| {nk} | {n} | {spans[len(spans) // 2]:.3f} |")
    if hist:
        nk = hist.most_common(1)[0][0]
        ks = next(ks for _, ks in graph if len(ks) == nk)
        names = collections.Counter(k[2][:90] for k in ks)
        print(f"\nKernels of one {nk}-kernel replay (one decode step):\n")
        print("| kernel | count |")
        print("|---|---|")
        for name, n in names.most_common():
            print(f"| `{name}` | {n} |")


if __name__ == "__main__":
    main()
