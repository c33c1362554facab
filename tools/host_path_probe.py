"""Host-array drop-in at BASELINE config-2 scale (diagnostic): run_alignment on 600 x 100k float64
frames held in numpy arrays (LMC:802-832 with the reference's calling convention), against the
transfer ceilings of the box (pinned H2D / D2H, pageable copies) and the cost of first-touching a
fresh output array of the same size.

    python tools/host_path_probe.py [--frames 600] [--points 100000] [--reps 3]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mc = importlib.import_module("livox-motion-compensation-sim_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    F, n = args.frames, args.points
    rng = np.random.default_rng(0)
    base = rng.standard_normal((n, 4)) * 30.0
    scans = [base + f * 1e-3 for f in range(F)]
    sim = mc.LiDARMotionSimulator({"duration": 120.0, "trajectory_type": "figure_eight", "max_speed": 12.0,
                                   "lidar_fps": 10})
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:F]
    out = {"frames": F, "points": n, "bytes_in": F * n * 32, "bytes_out": F * n * 32}
    t0 = time.perf_counter()
    a = np.empty((F * n, 4))
    a.fill(0.0)
    out["first_touch_out_s"] = time.perf_counter() - t0
    del a
    sim.run_alignment(scans[:2], tr, times[:2])
    walls = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        res = sim.run_alignment(scans, tr, times)
        walls.append(time.perf_counter() - t0)
        del res
    out["run_alignment_s"] = walls
    best = min(walls)
    out["Mpoints_s"] = F * n / best / 1e6
    out["GBs_in_plus_out"] = 64 * F * n / best / 1e9
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
