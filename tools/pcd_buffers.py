"""Does the ASCII-PCD write pass depend on which device buffer it writes into?  One process, one
batch, K text buffers allocated up front; every round encodes the batch into each buffer (order
shuffled) and the per-buffer medians of the codec kernels' time are printed (GPU box only).

    python tools/pcd_buffers.py [--buffers 4] [--rounds 9]
"""
from __future__ import annotations

import argparse
import json
import random
import statistics
import os
import sys
from ctypes import c_int64

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mcamd as mc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--buffers", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    ctx = mc.Context(0)
    counts = np.full(args.frames, args.points, np.int64)
    b = ctx.batch(counts)
    b.synth(seed=0, frame_id_base=1000)
    cap = int(counts.sum()) * 48
    bufs = [ctx.device_buffer(cap) for _ in range(args.buffers)]
    bpos = np.zeros(args.frames + 1, np.int64)
    ptr = mc._lib.ptr

    def pcd(buf):
        mc._lib.check(ctx.lib.mc_pcd_encode_batch(ctx.handle, b.handle, buf.ptr, cap, ptr(bpos, c_int64)),
                      "pcd_encode_batch")

    for buf in bufs:
        pcd(buf)
    ctx.sync()
    ctx.read_timing()
    times = {i: [] for i in range(len(bufs))}
    order = list(range(len(bufs)))
    rng = random.Random(1)
    for _ in range(args.rounds):
        rng.shuffle(order)
        for i in order:
            ctx.timing(True)
            for _ in range(args.reps):
                pcd(bufs[i])
            ctx.timing(False)
            times[i].append(ctx.read_timing()["codec_ms"] / args.reps * 1e3)
    out = {}
    for i in range(len(bufs)):
        out[i] = {"addr": hex(bufs[i].ptr.value), "median_us": statistics.median(times[i]), "min_us": min(times[i]),
                  "max_us": max(times[i])}
        print(f"buffer {i} {out[i]['addr']}: measure + write median {out[i]['median_us']:7.1f} us "
              f"(min {out[i]['min_us']:7.1f}, max {out[i]['max_us']:7.1f})", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
