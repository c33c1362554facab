"""Per-step timeline of the hot path from a rocprofv3 --kernel-trace CSV: for consecutive deskew
kernels, the idle gap between one kernel's end and the next one's start, and where the step's
k_prep ran relative to them.

    python tools/step_timeline.py gpurun_out/tl_x/**/run_kernel_trace.csv [--kernel k_deskew_points<1>]
Prints one JSON summary line (median / mean / max gap, prep duration, prep start relative to the
previous kernel's end) over the longest run of consecutive deskew kernels.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import statistics


def load(path):
    files = glob.glob(path, recursive=True)
    rows = []
    for fn in files:
        with open(fn) as f:
            rows += list(csv.DictReader(f))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_deskew_points<1")
    ap.add_argument("--label", default="")
    args = ap.parse_args()
    rows = load(args.trace)
    ev = []
    for r in rows:
        name = r["Kernel_Name"]
        kind = "main" if args.kernel in name else ("prep" if "k_prep" in name else None)
        if kind:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, r.get("Queue_Id")))
    ev.sort()
    mains = [e for e in ev if e[2] == "main"]
    preps = [e for e in ev if e[2] == "prep"]
    if len(mains) < 3:
        raise SystemExit("fewer than 3 deskew kernels in the trace")
    # the longest run of consecutive mains whose gaps stay below 1 ms (one timed block of steps)
    runs, cur = [], [mains[0]]
    for a, b in zip(mains, mains[1:]):
        if b[0] - a[1] < 1_000_000:
            cur.append(b)
        else:
            runs.append(cur)
            cur = [b]
    runs.append(cur)
    run = max(runs, key=len)
    gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(run, run[1:])]
    kern = [(e[1] - e[0]) / 1e3 for e in run]
    period = (run[-1][1] - run[0][0]) / 1e3 / len(run)
    # the prep that precedes each main (latest prep start before the main's start)
    prep_dur, prep_start_rel = [], []
    for a, b in zip(run, run[1:]):
        cand = [p for p in preps if p[0] <= b[0] and p[0] >= a[0] - 2_000_000]
        if cand:
            p = cand[-1]
            prep_dur.append((p[1] - p[0]) / 1e3)
            prep_start_rel.append((p[0] - a[1]) / 1e3)
    q = lambda v: {"median": statistics.median(v), "mean": statistics.mean(v), "min": min(v), "max": max(v)} if v else None
    print(json.dumps({"label": args.label, "steps": len(run), "kernel_us": q(kern), "gap_us": q(gaps),
                      "period_us": period, "period_over_kernel": period / statistics.mean(kern),
                      "prep_us": q(prep_dur), "prep_start_minus_prev_kernel_end_us": q(prep_start_rel),
                      "queues": sorted({str(e[3]) for e in run} | {str(p[3]) for p in preps})}))


if __name__ == "__main__":
    main()
