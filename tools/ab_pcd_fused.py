"""Interleaved A/B of the deskew -> PCD pipeline (mc_deskew_pcd vs mc_deskew + mc_pcd_encode_batch)
across library variants, one process, one device (GPU box only): bench.measure_deskew_pcd per
library and round, medians over rounds.

    python tools/ab_pcd_fused.py --libs build/variants/lib_pc0.so,build/variants/lib_pc1.so --modes pose_slerp,frame
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mcamd as mc  # noqa: E402
from tools.ab import setup  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--modes", default="pose_slerp,frame")
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    libs = [l for l in args.libs.split(",") if l]
    runs = {lib: setup(lib, args) for lib in libs}
    n = args.frames * args.points
    out = {}
    for mode in args.modes.split(","):
        res = {lib: [] for lib in libs}
        for _ in range(args.rounds):
            for lib in libs:
                ctx, (bt, bx), bo = runs[lib]
                res[lib].append(bench.measure_deskew_pcd(ctx, bx if mode == "frame" else bt, bo, mode, n, args.reps))
        for lib in libs:
            r = res[lib]
            med = {k: statistics.median(x[k2][k] for x in r) for k2, k in
                   (("separate", "deskew_kernel_us"), ("fused", "deskew_pcd_kernel_us"), ("fused", "write_ms"),
                    ("separate", "pcd_kernels_ms"))}
            fr = statistics.median(x["frac"] for x in r)
            name = os.path.basename(lib)
            out[f"{mode}/{name}"] = dict(med, frac=fr)
            print(f"{mode:10s} {name:16s} deskew {med['deskew_kernel_us']:7.1f} us  deskew_pcd {med['deskew_pcd_kernel_us']:7.1f} us "
                  f"(+{med['deskew_pcd_kernel_us'] - med['deskew_kernel_us']:5.1f})  write {med['write_ms'] * 1e3:7.1f} us  "
                  f"separate pcd {med['pcd_kernels_ms'] * 1e3:7.1f} us  fused frac {fr:.3f}", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ab_pcd_fused.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
