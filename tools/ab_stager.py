"""Interleaved A/B of the device stager pair (SoA f32 <-> AoS f64) across library variants, one
process, one device (GPU box only).  Also checks that every variant's round trip is bit-identical.

    make -C livox-motion-compensation-sim_amd/csrc variants VARIANTS="xcd:-DMC_XCD_STAGE=1 dealt:-DMC_XCD_STAGE=0"
    python tools/ab_stager.py --libs build/variants/lib_base.so,build/variants/lib_lds.so
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
import mcamd as mc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--replicas", type=int, default=1,
                    help="independent buffer sets per library, allocated alternately (page placement "
                         "moves streaming kernels by several percent, profiles/HISTORY_r1-r4.md section 8)")
    args = ap.parse_args()
    libs = [l for l in args.libs.split(",") if l]
    counts = np.full(args.frames, args.points, np.int64)
    counts[::7] -= 3                                    # ragged frames: partial groups and tiles
    n = int(counts.sum())
    runs = {}
    ctxs = {lib: mc.Context(0, lib_path=lib) for lib in libs}
    for r in range(args.replicas):
        for lib in libs:
            ctx = ctxs[lib]
            b = ctx.batch(counts)
            b.synth(seed=1, frame_id_base=1000)
            back = ctx.batch(counts)
            buf = ctx.device_buffer(n * 32)
            runs[(lib, r)] = (ctx, b, back, buf)
    ref = None
    for key, (ctx, b, back, buf) in runs.items():
        lib = key
        b.fetch_aos_device(buf)
        back.stage_aos_device(buf)
        ck = (b.checksum().tolist(), back.checksum().tolist())
        assert ck[0][:4] == ck[1][:4], (lib, ck)
        ref = ref or ck
        assert ck == ref, (lib, ck, ref)
    res = {key: {"soa_to_aos": [], "aos_to_soa": []} for key in runs}
    for _ in range(args.rounds):
        for lib, (ctx, b, back, buf) in runs.items():
            for name, fn in (("soa_to_aos", lambda: b.fetch_aos_device(buf)),
                             ("aos_to_soa", lambda: back.stage_aos_device(buf))):
                fn()
                ctx.sync()
                ctx.read_timing()
                ctx.timing(True)
                for _ in range(args.reps):
                    fn()
                ctx.sync()
                ctx.timing(False)
                t = ctx.read_timing()
                res[lib][name].append(t["layout_ms"] / t["layout_launches"] * 1e3)
    out = {}
    for lib in libs:
        out[os.path.basename(lib)] = {}
        for k in ("soa_to_aos", "aos_to_soa"):
            reps = [statistics.median(res[(lib, r)][k]) for r in range(args.replicas)]
            med = statistics.median(reps)
            out[os.path.basename(lib)][k] = {"median_us": med, "replica_medians_us": reps,
                                             "min_us": min(min(res[(lib, r)][k]) for r in range(args.replicas)),
                                             "frac_median": 48 * n / (med * 1e-6) / 8e12}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
