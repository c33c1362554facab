"""Interleaved A/B timing of library variants in ONE process on ONE device (GPU box only).

Each variant .so gets its own context and its own copy of the same workload; rounds alternate
between variants so clock / thermal drift hits all of them alike (cdna_hip_programming.md §5.4
rule 24).  Reports median and min of the hot kernel's HIP-event time per variant.

    make -C livox-motion-compensation-sim_amd/csrc variants
    python tools/ab.py --mode pose_slerp --libs build/variants/lib_base.so,build/variants/lib_w5.so
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import random
import statistics
import time
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mcamd as mc  # noqa: E402

BYTES = {"pose_slerp": 36, "imu": 36, "frame": 32}


def setup(lib, args):
    ctx = mc.Context(0, lib_path=lib)
    sim = mc.LiDARMotionSimulator({"duration": max(120.0, args.frames / 10.0), "trajectory_type": "figure_eight",
                                   "max_speed": 12.0, "lidar_fps": 10})
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:args.frames]
    counts = np.full(args.frames, args.points, np.int64)
    b_in = ctx.batch(counts, with_time=True)
    b_out = ctx.batch(counts)
    b_in.synth(seed=0, frame_id_base=1000)
    b_in.set_frame_times(times)
    b_in.set_frame_starts((times * 1e9).astype(np.int64))
    b_xyz = ctx.batch(counts)                     # frame mode: the reference's (N,4) points, no t_ns
    b_xyz.synth(seed=0, frame_id_base=1000)
    b_xyz.set_frame_times(times)
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    ts, g = mc.trajectory.imu_from_trajectory(tr, getattr(args, "imu_hz", 200.0))   # (setup is shared: ab_pcd_fused.py)
    ctx.set_imu(ts, g)
    return ctx, (b_in, b_xyz), b_out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default=",".join(sorted(glob.glob(os.path.join(ROOT, "build", "variants", "lib_*.so")))))
    ap.add_argument("--modes", default="pose_slerp,imu,frame")
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--grids", default="0", help="comma list of max-grid caps tried with every lib (0: one "
                                                  "workgroup per (sub-)tile)")
    ap.add_argument("--imu-hz", type=float, default=200.0, help="IMU sample rate of the workload (the reference's: 200)")
    ap.add_argument("--check", action="store_true",
                    help="after each mode, download every arm's output batch and compare it byte for byte with "
                         "the first arm's (variants that must not change results)")
    ap.add_argument("--replicas", type=int, default=1,
                    help="independent allocations (contexts) per library: where a batch's pages land moves a "
                         "kernel by up to ~10 %% (profiles/HISTORY_r1-r4.md section 8), so a variant is judged by the median "
                         "over its replicas")
    args = ap.parse_args()
    base_libs = [l for l in args.libs.split(",") if l]
    # replicas alternate across libraries so that no variant gets all the early (or late) allocations
    arms = [(lib, r) for r in range(args.replicas) for lib in base_libs]
    runs = {(f"{lib}#{r}" if args.replicas > 1 else lib): setup(lib, args) for lib, r in arms}
    libs = list(runs)
    grids = [int(g) for g in args.grids.split(",")]
    if grids != [0]:   # each (lib, grid) pair becomes its own arm, sharing the lib's workload
        runs = {f"{lib}@{g}": (*runs[lib], g) for lib in libs for g in grids}
    else:
        runs = {lib: (*runs[lib], 0) for lib in libs}
    variant = {arm: arm.split("#")[0] for arm in runs}   # arm -> library (replicas share one)
    libs = list(runs)
    n = args.frames * args.points
    out = {}
    for mode in args.modes.split(","):
        per = {lib: [] for lib in libs}
        wall = {lib: [] for lib in libs}
        order = list(libs)
        rng = random.Random(1)
        for _ in range(args.rounds):
            rng.shuffle(order)             # arm position within a round must not decide the result
            for lib in order:
                ctx, (bt, bx), bo, grid = runs[lib]
                bi = bx if mode == "frame" else bt
                ctx.set_max_grid(grid)
                for _ in range(3):
                    ctx.deskew(bi, bo, mode=mode)
                ctx.sync()
                t0 = time.perf_counter()          # wall pass: whole steps, no events inside
                for _ in range(args.steps):
                    ctx.deskew(bi, bo, mode=mode)
                ctx.sync()
                wall[lib].append((time.perf_counter() - t0) / args.steps * 1e6)
                ctx.read_timing()
                ctx.timing(True)                  # event pass: kernel time per launch
                for _ in range(args.steps):
                    ctx.deskew(bi, bo, mode=mode)
                ctx.sync()
                ctx.timing(False)
                t = ctx.read_timing()
                per[lib].append(t["main_ms"] / t["main_launches"] * 1e3)
                if hasattr(ctx.lib, "mc_timing_read_spans"):   # free the span slots: every timed launch stamps
                    ctx.read_timing_spans()
        if args.check:
            ref = None
            for lib in libs:
                ctx, (bt, bx), bo, grid = runs[lib]
                ctx.deskew(bx if mode == "frame" else bt, bo, mode=mode)
                ctx.sync()
                cols = np.stack([np.ascontiguousarray(c) for c in bo.download_columns()[:4]])
                if ref is None:
                    ref = cols
                    continue
                diff = int(np.count_nonzero(cols.view(np.uint32) != ref.view(np.uint32)))
                print(f"{mode:10s} {os.path.basename(lib):22s} output vs {os.path.basename(libs[0])}: "
                      f"{'identical' if diff == 0 else f'{diff} values differ'}", flush=True)
                if diff:
                    raise SystemExit(f"{mode}: {lib} output differs")
            del ref
        for lib in libs:
            v = per[lib]
            med = statistics.median(v)
            wmed = statistics.median(wall[lib])
            name = os.path.basename(lib)
            out[f"{mode}/{name}"] = {"median_us": med, "min_us": min(v), "step_wall_us": wmed,
                                     "GBs": BYTES[mode] * n / (med * 1e-6) / 1e9}
            print(f"{mode:10s} {name:22s} kernel median {med:7.1f} us  min {min(v):7.1f} us  "
                  f"{BYTES[mode] * n / (med * 1e-6) / 1e9:6.0f} GB/s | step wall {wmed:7.1f} us "
                  f"(+{wmed - med:5.1f})", flush=True)
        if args.replicas > 1:   # per variant: median over its replicas' medians
            for var in dict.fromkeys(variant.values()):
                meds = [statistics.median(per[a]) for a in libs if variant[a] == var]
                name = os.path.basename(var)
                out[f"{mode}/{name}/replicas"] = {"median_us": statistics.median(meds), "replica_medians_us": meds}
                print(f"{mode:10s} {name:22s} over {len(meds)} replicas: median {statistics.median(meds):7.1f} us "
                      f"(replicas {', '.join(f'{m:.1f}' for m in meds)})", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ab.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
