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
    ctx = sim.context
    from ctypes import c_double, c_int64
    ptr = mc._lib.ptr
    counts = np.full(F, n, np.int64)
    lds = np.full(F, 4, np.int64)
    offs = np.concatenate([[0], np.cumsum(counts)])
    fp = np.fromiter((f.__array_interface__["data"][0] for f in scans), np.uintp, F)
    pref = np.zeros((F * n, 4))                                       # pre-faulted, reused output
    op = (pref.__array_interface__["data"][0] + 32 * offs[:-1]).astype(np.uintp)
    t = np.ascontiguousarray(times, np.float64)
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])

    def direct():
        mc._lib.check(ctx.lib.mc_align_frames_host_f64(ctx.handle, F, fp.ctypes.data, ptr(counts, c_int64),
                                                       ptr(lds, c_int64), ptr(t, c_double), mc._lib.MC_POSE_SEARCHSORTED,
                                                       op.ctypes.data), "align")
    ref = None
    first = True
    for rows in ("",):
        walls, pre = [], []
        res = None
        for _ in range(args.reps):
            res = None                                    # the previous result is freed first
            t0 = time.perf_counter()
            res = sim.run_alignment(scans, tr, times)
            walls.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            direct()                                      # into a pre-faulted pageable array
            pre.append(time.perf_counter() - t0)
        same = None
        if ref is None:
            ref = [r.copy() for r in res[:5]]
        else:
            same = all(np.array_equal(a, b) for a, b in zip(ref, res[:5]))
        res = None
        out[f"rows_{rows or 'default'}"] = {
            "run_alignment_s": walls, "Mpoints_s": F * n / min(walls) / 1e6,
            "Mpoints_s_steady_median": F * n / float(np.median(walls[1:] if len(walls) > 1 else walls)) / 1e6,
            "first_call_s" if first else "first_call_s_pool_warm": walls[0],
            "pageable_prefaulted_out_s": pre, "pageable_prefaulted_Mpoints_s": F * n / min(pre) / 1e6,
            "equal_to_first": same}
        first = False
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
