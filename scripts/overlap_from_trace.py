#!/usr/bin/env python3
"""How much of the verification kernels' time overlaps other kernels (rocprofv3 kernel trace).

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 bench.py --steps 3
    python scripts/overlap_from_trace.py OUT/.../run_kernel_trace.csv [--match grad_partial,grad_segment]

For every dispatch whose name matches, the part of its [start, end) interval covered by at least
one dispatch of a non-matching kernel (on any queue) counts as overlapped.  Prints per-name totals
and the overall overlapped fraction: the verification pass running on the side stream while the
backward's GEMMs still run shows up as a high fraction; a serial tail as ~0.
"""
import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="grad_partial_kernel,grad_segment_kernel,grad_summary_kernel,hist_kernel,"
                                       "quantile_kernel,moments_partial_kernel,moments_final_kernel,zscore_kernel")
    args = ap.parse_args()
    keys = [k for k in args.match.split(",") if k]
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            s = int(r.get("Start_Timestamp") or r.get("BeginNs") or 0)
            e = int(r.get("End_Timestamp") or r.get("EndNs") or 0)
            if e > s:
                rows.append((name, s, e))
    rows.sort(key=lambda t: t[1])
    mine = [(n, s, e) for n, s, e in rows if any(k in n for k in keys)]
    other = [(s, e) for n, s, e in rows if not any(k in n for k in keys)]
    # merged intervals of the other kernels
    merged = []
    for s, e in sorted(other):
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    import bisect
    starts = [m[0] for m in merged]
    per = defaultdict(lambda: [0, 0, 0])   # name -> [count, total ns, overlapped ns]
    for n, s, e in mine:
        i = max(0, bisect.bisect_right(starts, s) - 1)
        ov = 0
        while i < len(merged) and merged[i][0] < e:
            a, b = max(s, merged[i][0]), min(e, merged[i][1])
            if b > a:
                ov += b - a
            i += 1
        key = next(k for k in keys if k in n)
        per[key][0] += 1
        per[key][1] += e - s
        per[key][2] += ov
    tot = sum(v[1] for v in per.values())
    ovl = sum(v[2] for v in per.values())
    out = {"kernels": {k: {"dispatches": v[0], "total_us": round(v[1] / 1e3, 1), "overlapped_us": round(v[2] / 1e3, 1),
                           "overlapped_frac": round(v[2] / v[1], 3) if v[1] else 0.0} for k, v in per.items()},
           "total_us": round(tot / 1e3, 1), "overlapped_us": round(ovl / 1e3, 1),
           "overlapped_frac": round(ovl / tot, 3) if tot else 0.0}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
