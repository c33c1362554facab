"""Is the deskew kernels' HBM rate helped by the 256 MB Infinity Cache (MALL) re-serving the previous
step's buffers?  One step reads 1.2 GB and writes 0.96 GB (600 x 100k, SLERP), so at most
256 MB / 2.16 GB of a step could be re-served; this A/B measures it (GPU box only):

  same      every step on buffer set A (the bench's pattern)
  pp2       steps alternate between two independent sets A, B (4.3 GB working set)
  pp4       four sets (8.6 GB)
  flush     set A, but a 2 GB streaming copy of unrelated buffers runs before every step
            (untimed; the kernel's events time the deskew kernel only)
  fread     set A after a read-only 2 GB pass (mc_batch_checksum of an unrelated batch): the
            Infinity Cache left full of clean lines
  fwrite    set A after a write-only 2 GB pass (mc_batch_synth of that batch): left full of dirty
            lines, whose write-back lands in the next kernel
  f256      as flush, with a 256 MB copy (the Infinity Cache's size) instead of 2 GB
  fslerp    set A after a SLERP deskew of the unrelated 100 M-point batch (1.6 GB written with the
            production SLERP store policy)
  fidle     set A after 2 ms of host sleep (the device idles between steps)

--libs runs every arm for several library builds in one process (one context per library), e.g.
the production SLERP store policy (sc1 write-through) against a build with nt stores
(-DMC_STORE_POINTS=1): which arm costs which store policy names the mechanism.

Each arm: HIP events on every deskew launch (hipExtLaunchKernel start/stop); arms interleave over
rounds in one process.  Each set is a separate allocation, so placement differs per set: the
per-set medians are reported too.

    python tools/pingpong.py --modes pose_slerp,imu,frame --rounds 5 --steps 16
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mcamd as mc  # noqa: E402

BYTES = {"pose_slerp": 36, "imu": 36, "frame": 32}


def make_set(ctx, counts, times, seed):
    b_in = ctx.batch(counts, with_time=True)
    b_in.synth(seed=seed, frame_id_base=1000)
    b_in.set_frame_times(times)
    b_in.set_frame_starts((times * 1e9).astype(np.int64))
    b_xyz = ctx.batch(counts)
    b_xyz.synth(seed=seed, frame_id_base=1000)
    b_xyz.set_frame_times(times)
    return {"in": b_in, "xyz": b_xyz, "out": ctx.batch(counts)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="pose_slerp,imu,frame")
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pingpong.json"))
    ap.add_argument("--libs", default="", help="comma list of library builds (default: the in-tree one)")
    ap.add_argument("--arms", default="same,pp2,pp4,flush,fread,fwrite")
    args = ap.parse_args()
    libs = [l for l in args.libs.split(",") if l] or [None]
    res = {}
    for lib in libs:
        run_lib(args, lib, res)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)


def run_lib(args, lib, res):
    name = os.path.basename(lib) if lib else "in-tree"
    ctx = mc.Context(0, lib_path=lib) if lib else mc.Context(0)
    sim = mc.LiDARMotionSimulator({"duration": 120.0, "trajectory_type": "figure_eight", "max_speed": 12.0,
                                   "lidar_fps": 10})
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:args.frames]
    counts = np.full(args.frames, args.points, np.int64)
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    ts, g = mc.trajectory.imu_from_trajectory(tr, 200.0)
    ctx.set_imu(ts, g)
    sets = [make_set(ctx, counts, times, s) for s in range(4)]
    n = int(counts.sum())
    flush_a = ctx.device_buffer(2 << 30)
    flush_b = ctx.device_buffer(2 << 30)
    sweep = ctx.batch(np.full(1000, 100_000, np.int64), with_time=True)   # 100 M points x 5 columns = 2 GB
    sweep.synth(seed=99, frame_id_base=0)
    sweep.set_frame_times(sim.lidar_times()[:1000])
    sweep_out = ctx.batch(sweep.counts)
    all_arms = {"same": [0], "pp2": [0, 1], "pp4": [0, 1, 2, 3], "flush": [0], "fread": [0], "fwrite": [0],
                "f256": [0], "fslerp": [0], "fidle": [0]}
    arms = {a: all_arms[a] for a in args.arms.split(",")}
    for mode in args.modes.split(","):
        key = "xyz" if mode == "frame" else "in"
        per = {a: [] for a in arms}
        per_set = {a: {s: [] for s in arms[a]} for a in arms}
        for rnd in range(args.rounds):
            for arm, use in arms.items():
                for k in range(4):                       # warm every set of the arm
                    s = sets[use[k % len(use)]]
                    ctx.deskew(s[key], s["out"], mode=mode)
                ctx.sync()
                ctx.read_timing()
                for i in range(args.steps):
                    s_id = use[i % len(use)]
                    s = sets[s_id]
                    if arm == "flush":                  # evict the MALL: 2 GB D2D copy, untimed
                        mc._lib.check(ctx.lib.mc_memcpy_d2d(ctx.handle, flush_b.ptr, flush_a.ptr, flush_a.nbytes),
                                      "memcpy_d2d")
                    elif arm == "fread":                # 2 GB read-only sweep (clean lines)
                        sweep.checksum()
                    elif arm == "fwrite":               # 2 GB write-only sweep (dirty lines)
                        sweep.synth(seed=99, frame_id_base=0)
                        ctx.sync()
                    elif arm == "f256":                 # 256 MB D2D copy
                        mc._lib.check(ctx.lib.mc_memcpy_d2d(ctx.handle, flush_b.ptr, flush_a.ptr, 256 << 20),
                                      "memcpy_d2d")
                    elif arm == "fslerp":               # SLERP deskew of another 100 M points
                        ctx.deskew(sweep, sweep_out, mode="pose_slerp")
                    elif arm == "fidle":                # the device idles 2 ms
                        ctx.sync()
                        time.sleep(0.002)
                    ctx.timing(True)
                    ctx.deskew(s[key], s["out"], mode=mode)
                    ctx.timing(False)
                    ctx.sync()
                    t = ctx.read_timing()
                    us = t["main_ms"] / max(t["main_launches"], 1) * 1e3
                    per[arm].append(us)
                    per_set[arm][s_id].append(us)
        for arm in arms:
            med = statistics.median(per[arm])
            res[f"{name}/{mode}/{arm}"] = {"median_us": med, "min_us": min(per[arm]), "max_us": max(per[arm]),
                                   "frac": BYTES[mode] * n / (med * 1e-6) / 8e12,
                                   "per_set_median_us": {str(s): statistics.median(v) for s, v in per_set[arm].items()}}
            print(f"{name:16s} {mode:10s} {arm:6s} median {med:7.1f} us  ({BYTES[mode] * n / (med * 1e-6) / 1e9:6.0f} GB/s)  "
                  f"per set: {', '.join(f'{s}:{statistics.median(v):.1f}' for s, v in per_set[arm].items())}",
                  flush=True)
    sweep.close()
    sweep_out.close()
    flush_a.close()
    flush_b.close()
    for s in sets:
        for b in s.values():
            b.close()


if __name__ == "__main__":
    main()
