"""The bench line's roofline kernel time, recomputed from a rocprofv3 kernel trace of the same run.

bench.py times its roofline kernel on every `every`-th of the K timed steps: since round 4 by the
launch's own workgroup span (first workgroup start to last workgroup end on the device wall clock,
mc_timing_read_spans), with the HIP events of the same launches beside it (their start marker also
holds the ~5 us dispatch gap ahead of the launch).  rocprofv3's --stats average mixes
in every other launch of that kernel in the process (the 250 ms spin-up, mc_tune_order's candidate
orders, the warmup steps), so it does not reproduce the line (What's weak 2).  This
tool picks the timed window out of the kernel trace of the profiled bench command itself — in
pipeline issue the K timed steps are one k_prep, K - 1 launches of the fused kernel and one plain
launch, the only such run of exactly K - 1 fused launches in the process (spin-up runs have 24,
warmup runs W - 1, tuning runs 1 and `launches` - 1) — and averages the same sampled launches.

    python tools/roofline_from_trace.py --trace <dir with *kernel_trace.csv> --bench <bench json> \
        [--out summary.json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys

FUSED = {"pose_slerp": "k_deskew_points<1, true, false>", "imu": "k_deskew_points<2, true, false>",
         "frame": "k_deskew_frame_next"}
PLAIN = {"pose_slerp": "k_deskew_points<1, false, false>", "imu": "k_deskew_points<2, false, false>",
         "frame": "k_deskew_frame("}


def load_trace(path: str):
    files = [path] if os.path.isfile(path) else sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"),
                                                                 recursive=True))
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {path}")
    rows = []
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                rows.append({"name": r["Kernel_Name"], "start": int(r["Start_Timestamp"]),
                             "end": int(r["End_Timestamp"]),
                             "pid": f, "queue": r.get("Queue_Id", "")})
    rows.sort(key=lambda r: (r["pid"], r["start"]))
    return rows, files


def timed_window(rows, mode: str, steps: int):
    """Indices (into rows) of the K timed steps' kernels: the run of exactly K - 1 fused launches
    between a k_prep and a plain launch."""
    fused, plain = FUSED[mode], PLAIN[mode]
    found = []
    i = 0
    while i < len(rows):
        if fused in rows[i]["name"]:
            j = i
            while j < len(rows) and fused in rows[j]["name"]:
                j += 1
            n = j - i
            prev_prep = i > 0 and "k_prep" in rows[i - 1]["name"]
            next_plain = j < len(rows) and plain in rows[j]["name"]
            if n == steps - 1 and prev_prep and next_plain:
                found.append(list(range(i, j + 1)))
            i = j
        else:
            i += 1
    return found


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--bench", required=True, help="the JSON line bench.py printed in the profiled run")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    with open(a.bench) as f:
        line = json.loads([ln for ln in f if ln.strip().startswith("{")][-1])
    mode = line["config"]["mode"]
    steps = int(line["steps"])
    every = 10 if steps >= 50 else 5
    rows, files = load_trace(a.trace)
    wins = timed_window(rows, mode, steps)
    if len(wins) != 1:
        raise SystemExit(f"expected one timed window of {steps - 1} fused launches, found {len(wins)}")
    win = wins[0]
    dur = [(rows[k]["end"] - rows[k]["start"]) / 1e3 for k in win]   # ns -> us
    sampled = [dur[i] for i in range(steps) if i % every == every // 2]
    fused_all = [(r["end"] - r["start"]) / 1e3 for r in rows if FUSED[mode] in r["name"]]
    bench_us = line["roofline"]["kernel_avg_us"]
    trace_us = sum(sampled) / len(sampled)
    bpp, n = line["roofline"]["bytes_per_point"], line["roofline"]["points_per_launch"]
    out = {
        "mode": mode, "kernel": FUSED[mode], "steps": steps, "sampled_every": every,
        "trace_files": [os.path.relpath(f) for f in files],
        "timed_window_launches": len(win),
        "sampled_steps_us": [round(x, 2) for x in sampled],
        "trace_sampled_avg_us": trace_us,
        "trace_all_timed_steps_avg_us": sum(dur) / len(dur),
        "bench_line_kernel_avg_us": bench_us,
        "trace_vs_bench": trace_us / bench_us - 1.0,
        "bench_kernel_each_us": line["roofline"].get("kernel_each_us"),
        "bench_minus_trace_each_us": ([round(e - t, 2) for e, t in zip(line["roofline"]["kernel_each_us"], sampled)]
                                      if line["roofline"].get("kernel_each_us") else None),
        "bench_events_each_us": line["roofline"].get("events_each_us"),
        "events_minus_trace_each_us": ([round(e - t, 2) for e, t in zip(line["roofline"]["events_each_us"], sampled)]
                                       if line["roofline"].get("events_each_us") else None),
        "bench_kernel_time": line["roofline"].get("kernel_time"),
        "frac_from_trace": bpp * n / (trace_us * 1e-6) / 1e9 / line["roofline"]["peak"],
        "frac_bench_line": line["roofline"]["frac"],
        "all_launches_of_kernel_avg_us": sum(fused_all) / len(fused_all),
        "all_launches_of_kernel": len(fused_all),
        "note": "the sampled steps are the bench's own HIP-event steps (i % every == every // 2 of the K timed steps); "
                "all_launches_* is what rocprofv3 --stats averages (spin-up, tuning, warmup included)",
    }
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    return 0 if abs(out["trace_vs_bench"]) <= 0.01 else 1


if __name__ == "__main__":
    sys.exit(main())
