"""Placement study (profiles/HISTORY_r1-r4.md §8): identical frame-mode kernels on R independent allocations of the
same 600 x 100k workload ("replicas") run at two distinct speeds.  Each replica runs K kernels in
turn (replica 0 x K, replica 1 x K, ...), so under ``rocprofv3 --pmc`` dispatch order maps a
counter row to its replica; HIP events give each replica's kernel time in the same run.

    rocprofv3 -E tools/pmc/tcc_channels.yaml --pmc MC_RD_I0 ... -- python3 tools/placement_pmc.py
    python3 tools/placement_pmc.py --parse <rocprof dir> --times gpurun_out/placement_times.json

Without --parse: runs the replicas and writes their kernel times (--times).  With --parse: reads
the counter CSV of that run and prints, per replica, the kernel time and every counter's median.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(args):
    import mcamd as mc
    ctx = mc.Context(0)
    sim = mc.LiDARMotionSimulator({"duration": 120.0, "trajectory_type": "figure_eight", "max_speed": 12.0,
                                   "lidar_fps": 10})
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:args.frames]
    counts = np.full(args.frames, args.points, np.int64)
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    reps = []
    for r in range(args.replicas):
        b = ctx.batch(counts)
        b.synth(seed=r, frame_id_base=1000)
        b.set_frame_times(times)
        reps.append((b, ctx.batch(counts)))
    for b, o in reps:                     # warm every replica once (not counted: --warm)
        ctx.deskew(b, o, mode=args.mode)
    ctx.sync()
    out = []
    for b, o in reps:
        ctx.read_timing()
        ctx.timing(True)
        for _ in range(args.k):
            ctx.deskew(b, o, mode=args.mode)
        ctx.sync()
        ctx.timing(False)
        t = ctx.read_timing()
        out.append(t["main_ms"] / t["main_launches"] * 1e3)
    print(json.dumps({"kernel_us": out}))
    if args.times:
        with open(args.times, "w") as f:
            json.dump({"kernel_us": out, "replicas": args.replicas, "k": args.k, "mode": args.mode}, f)


def parse(args):
    kern = {"frame": "k_deskew_frame", "pose_slerp": "k_deskew_points<1", "imu": "k_deskew_points<2"}[args.mode]
    rows = []
    for fn in glob.glob(os.path.join(args.parse, "**", "*counter_collection*.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(fn)) if kern in r["Kernel_Name"]]
    disp = sorted({int(r["Dispatch_Id"]) for r in rows})
    # first R dispatches are the warm-up launches; then K per replica
    t = json.load(open(args.times))
    R, K = t["replicas"], t["k"]
    body = disp[R:]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        d = int(r["Dispatch_Id"])
        if d in body:
            per[body.index(d) // K][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = []
    for rep in range(R):
        c = {k: statistics.median(v) for k, v in sorted(per[rep].items())}
        res.append({"replica": rep, "kernel_us": t["kernel_us"][rep], "counters": c})
        print(json.dumps(res[-1]))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=6)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--mode", default="frame")
    ap.add_argument("--times", default="")
    ap.add_argument("--parse", default="")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    parse(args) if args.parse else run(args)


if __name__ == "__main__":
    main()
