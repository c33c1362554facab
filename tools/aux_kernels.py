"""Drive the kernels around the hot path a few times each on the bench workload (GPU box only),
for rocprofv3 counter passes (tools/pmc_traffic.py --aux).  Prints one JSON line with the
algorithmic HBM bytes of one launch of each kernel.

    python tools/aux_kernels.py [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from ctypes import c_int64, c_uint64

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mcamd as mc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    ctx = mc.Context()
    counts = np.full(args.frames, args.points, np.int64)
    n = int(counts.sum())
    b = ctx.batch(counts)
    b.synth(seed=0, frame_id_base=1000)
    src = ctx.device_buffer(n * 32)
    ptr = mc._lib.ptr
    for _ in range(args.reps):
        b.fetch_aos_device(src)                # k_soa_to_aos
    for _ in range(args.reps):
        b.stage_aos_device(src)                # k_aos_to_soa
    pos = mc.codecs.lvx_layout(counts)
    ids = np.arange(args.frames, dtype=np.uint64)
    ts = (np.arange(args.frames) * 100_000_000).astype(np.uint64)
    out = ctx.device_buffer(int(pos[-1]))
    for _ in range(args.reps):                 # from the batch's float32 columns (16 B / point read)
        mc._lib.check(ctx.lib.mc_lvx_encode_batch(ctx.handle, b.handle, ptr(ids, c_uint64), ptr(ts, c_uint64),
                                                  out.ptr, int(pos[-1])))
    out.close()
    cap = n * 48
    out = ctx.device_buffer(cap)
    bpos = np.zeros(args.frames + 1, np.int64)
    for _ in range(args.reps):
        mc._lib.check(ctx.lib.mc_pcd_encode_batch(ctx.handle, b.handle, out.ptr, cap, ptr(bpos, c_int64)))
    out.close()
    rng = np.random.default_rng(7)
    E = 29_000
    env = np.column_stack([rng.uniform(-200, 200, E), rng.uniform(-200, 200, E), rng.uniform(-25, 70, E),
                           rng.uniform(0, 1, E)])
    cfg = dict(mc.default_config(), duration=120.0, trajectory_type="figure_eight", max_speed=12.0, lidar_fps=10)
    sim = mc.LiDARMotionSimulator(cfg, context=ctx)
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()
    ctx.set_environment(env)
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    scans = None
    for _ in range(args.reps):
        scans = ctx.scan(times, dict(cfg, lidar_range_noise=0.0), out=scans)
    ctx.sync()
    F = len(times)
    tiles, Fp = (E + 1023) // 1024, (F + 7) // 8 * 8
    bits = tiles * (Fp // 8) * 256 * 4                         # pass-1 visibility words
    poses = 96 * F                                             # R (9) + t (3) float64 per frame
    n_out = int(scans.n_points)
    alg = {
        "k_soa_to_aos": 48 * n, "k_aos_to_soa": 48 * n,
        # the points in, the file out but its 88-byte header (the frame headers too: round 5)
        "k_lvx_packages": 16 * n + int(pos[-1]) - 88,
        "k_pcd_measure": 16 * n, "k_pcd_write": 16 * n + int(bpos[-1]),
        # scene x, y, z once + the poses once + the visibility words + the per-(tile, frame) counts
        "k_scan_count": 24 * E + poses + bits + 4 * tiles * Fp,
        # ... + the offsets (8 B) + per-frame visible counts, and per emitted point its float64
        # intensity (8 B) and its float32 output row (16 B)
        "k_scan_emit": 24 * E + poses + bits + 8 * tiles * Fp + 8 * F + 24 * n_out,
    }
    print(json.dumps({"algorithmic_bytes_per_launch": alg, "points": n, "scene": E, "frames_scanned": len(times),
                      "note": "scan kernels: the scene (24 B/pt of x,y,z columns) and the frame poses (96 B) "
                              "are read once from HBM and then re-read from L2; algorithmic = those + the "
                              "visibility words, counts / offsets and output"}))


if __name__ == "__main__":
    main()
