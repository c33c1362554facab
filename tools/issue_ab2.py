"""Step-issue A/B in one process (GPU box only): per-step wall time of the headline SLERP step over
BASELINE config 2 (600 x 100k) issued as
  call     K plain mc_deskew calls (prep any-order packet + kernel), no timing events
  call_ev  the same with hipExtLaunchKernel events on every 5th kernel (bench.py's protocol)
  g1       K calls of a cached one-step HIP graph (mc_deskew_steps(1))
  gK       one replay of a K-step graph (mc_deskew_steps(K))
for K = 20 (the driver's bench) and K = 100, interleaved over rounds; kernel time by events.

    python tools/issue_ab2.py --rounds 4
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--mode", default="pose_slerp")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "issue_ab2.json"))
    args = ap.parse_args()
    ctx = mc.Context(0)
    sim = mc.LiDARMotionSimulator({"duration": 120.0, "trajectory_type": "figure_eight", "max_speed": 12.0,
                                   "lidar_fps": 10})
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:600]
    counts = np.full(600, 100_000, np.int64)
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    ts, gyro = mc.trajectory.imu_from_trajectory(tr, 200.0)
    ctx.set_imu(ts, gyro)
    b_in = ctx.batch(counts, with_time=True)
    b_in.synth(seed=0, frame_id_base=1000)
    b_in.set_frame_times(times)
    b_in.set_frame_starts((times * 1e9).astype(np.int64))
    b_out = ctx.batch(counts)
    m = args.mode

    def timed(fn):
        ctx.sync()
        t0 = time.perf_counter()
        fn()
        ctx.sync()
        return time.perf_counter() - t0

    res = {}
    for _ in range(3):
        ctx.deskew(b_in, b_out, mode=m)
    for rnd in range(args.rounds):
        for K in (20, 100):
            # call
            ctx.deskew(b_in, b_out, mode=m)
            res.setdefault(f"call K={K}", []).append(timed(lambda: [ctx.deskew(b_in, b_out, mode=m)
                                                                    for _ in range(K)]) / K * 1e6)

            def call_ev():
                for i in range(K):
                    s = i % 5 == 2
                    if s:
                        ctx.timing(True)
                    ctx.deskew(b_in, b_out, mode=m)
                    if s:
                        ctx.timing(False)
            ctx.read_timing()
            res.setdefault(f"call_ev K={K}", []).append(timed(call_ev) / K * 1e6)
            t = ctx.read_timing()
            res.setdefault(f"kernel_ev K={K}", []).append(t["main_ms"] / max(t["main_launches"], 1) * 1e3)
            # one-step graph per call
            ctx.deskew_steps(b_in, b_out, 1, mode=m, prepare=True)
            ctx.deskew_steps(b_in, b_out, 1, mode=m)
            res.setdefault(f"g1 K={K}", []).append(timed(lambda: [ctx.deskew_steps(b_in, b_out, 1, mode=m)
                                                                  for _ in range(K)]) / K * 1e6)
            # K-step graph
            ctx.deskew_steps(b_in, b_out, K, mode=m, prepare=True)
            res.setdefault(f"gK K={K}", []).append(timed(lambda: ctx.deskew_steps(b_in, b_out, K, mode=m)) / K * 1e6)
        print(f"round {rnd} done", flush=True)
    summ = {k: {"median_us": statistics.median(v), "min_us": min(v), "all": v} for k, v in res.items()}
    for k, v in summ.items():
        print(f"{k:16s} median {v['median_us']:8.1f} us  min {v['min_us']:8.1f}")
    with open(args.out, "w") as f:
        json.dump(summ, f)


if __name__ == "__main__":
    main()
