"""Interleaved, order-shuffled A/B of the LVX and ASCII-PCD encoders across library variants, one
process, one device (GPU box only).  Each arm encodes the same device (N,4) f64 cloud; outputs of
every arm are checked byte-identical to the first arm's.

    make -C livox-motion-compensation-sim_amd/csrc variants VARIANTS="a:-DMC_XCD_CODEC=1 b:-DMC_XCD_CODEC=0"
    python tools/ab_codecs.py --libs build/variants/lib_a.so,build/variants/lib_b.so
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
from ctypes import c_int64, c_uint64

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mcamd as mc  # noqa: E402


def setup(lib, counts, source="aos", flush_on=False):
    ctx = mc.Context(0, lib_path=lib)
    b = ctx.batch(counts)
    b.synth(seed=0, frame_id_base=1000)
    src = None
    if source == "aos":
        src = ctx.device_buffer(int(counts.sum()) * 32)
        b.fetch_aos_device(src)
    F = len(counts)
    pos = mc.codecs.lvx_layout(counts)
    lvx_out = ctx.device_buffer(int(pos[-1]))
    cap = int(counts.sum()) * 48
    pcd_out = ctx.device_buffer(cap)
    ids = np.arange(F, dtype=np.uint64)
    ts = (np.arange(F) * 100_000_000).astype(np.uint64)
    bpos = np.zeros(F + 1, np.int64)
    ptr = mc._lib.ptr

    def lvx():
        if source == "batch":   # the batch's own float32 columns (mc_lvx_encode_batch)
            mc._lib.check(ctx.lib.mc_lvx_encode_batch(ctx.handle, b.handle, ptr(ids, c_uint64), ptr(ts, c_uint64),
                                                      lvx_out.ptr, int(pos[-1])), "lvx_encode_batch")
            return
        mc._lib.check(ctx.lib.mc_lvx_encode(ctx.handle, src.ptr, 4, F, ptr(counts, c_int64), ptr(ids, c_uint64),
                                            ptr(ts, c_uint64), None, lvx_out.ptr, int(pos[-1])), "lvx_encode")

    def pcd():
        if source == "batch":
            mc._lib.check(ctx.lib.mc_pcd_encode_batch(ctx.handle, b.handle, pcd_out.ptr, cap, ptr(bpos, c_int64)),
                          "pcd_encode_batch")
            return
        mc._lib.check(ctx.lib.mc_pcd_encode(ctx.handle, src.ptr, 4, F, ptr(counts, c_int64), pcd_out.ptr, cap,
                                            ptr(bpos, c_int64)), "pcd_encode")

    flush_buf = ctx.batch(np.full(len(counts), int(counts.max()), np.int64), with_time=True) if flush_on else None

    def flush():
        flush_buf.checksum()

    return {"ctx": ctx, "batch": b, "lvx": lvx, "pcd": pcd, "flush": flush, "lvx_out": lvx_out, "pcd_out": pcd_out, "bpos": bpos,
            "lvx_bytes": int(pos[-1])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--flush", action="store_true",
                    help="a checksum pass over a 2 GB scratch buffer before every timed call (the previous "
                         "call's dirty lines are written back outside the timed kernels)")
    ap.add_argument("--no-check", action="store_true", help="skip the byte-identity check (diagnostic builds)")
    ap.add_argument("--source", default="aos", choices=["aos", "batch"],
                    help="encode from a device (N,4) float64 AoS array or from the batch's float32 columns")
    ap.add_argument("--replicas", type=int, default=1,
                    help="independent allocations per library (placement moves a kernel by a few %%); a "
                         "library's figure is the median over its replicas' medians")
    args = ap.parse_args()
    base_libs = [l for l in args.libs.split(",") if l]
    counts = np.full(args.frames, args.points, np.int64)
    # replicas alternate across libraries so that no variant gets all the early (or late) allocations
    libs = [f"{lib}#{r}" if args.replicas > 1 else lib for r in range(args.replicas) for lib in base_libs]
    arms = {arm: setup(arm.split("#")[0], counts, args.source, args.flush) for arm in libs}
    times = {lib: {"lvx": [], "pcd": []} for lib in libs}
    order = list(libs)
    rng = random.Random(1)
    for _ in range(args.rounds):
        rng.shuffle(order)
        for lib in order:
            a = arms[lib]
            for name in ("lvx", "pcd"):
                a[name]()
                a["ctx"].read_timing()
                a["ctx"].timing(True)
                for _ in range(args.reps):
                    if args.flush:
                        a["flush"]()
                    a[name]()
                a["ctx"].timing(False)
                times[lib][name].append(a["ctx"].read_timing()["codec_ms"] / args.reps * 1e3)
    # byte-identical outputs across arms (libraries named lib_diag* are diagnostics: reported, not enforced)
    ref = arms[libs[0]]
    bad = []
    for lib in ([] if args.no_check else libs[1:]):
        a = arms[lib]
        for key, nbytes in (("lvx_out", ref["lvx_bytes"]), ("pcd_out", int(ref["bpos"][-1]))):
            los = range(0, nbytes, 64 << 20)   # the whole file / text
            same = True
            for lo in los:
                n = min(64 << 20, nbytes - lo)
                x = np.empty(n, np.uint8)
                y = np.empty(n, np.uint8)
                mc._lib.check(ref["ctx"].lib.mc_memcpy_d2h(ref["ctx"].handle, x.ctypes.data, ref[key].ptr.value + lo, n))
                mc._lib.check(a["ctx"].lib.mc_memcpy_d2h(a["ctx"].handle, y.ctypes.data, a[key].ptr.value + lo, n))
                same = same and np.array_equal(x, y)
            name = os.path.basename(lib)
            print(f"{name:22s} {key}: {'identical' if same else 'DIFFERS'}", flush=True)
            if not same and not name.startswith("lib_diag"):
                bad.append((name, key))
    out = {}
    for lib in libs:
        name = os.path.basename(lib)
        out[name] = {k: {"median_us": statistics.median(v), "min_us": min(v)} for k, v in times[lib].items()}
        print(f"{name:22s} lvx median {out[name]['lvx']['median_us']:8.1f} us   pcd (measure+write) median "
              f"{out[name]['pcd']['median_us']:8.1f} us", flush=True)
    if args.replicas > 1:
        for lib in base_libs:
            name = os.path.basename(lib)
            per = {k: [out[f"{name}#{r}"][k]["median_us"] for r in range(args.replicas)] for k in ("lvx", "pcd")}
            out[name] = {k: {"median_us": statistics.median(v), "replica_medians_us": v} for k, v in per.items()}
            lvx_reps = ", ".join(f"{x:.1f}" for x in per["lvx"])
            pcd_reps = ", ".join(f"{x:.1f}" for x in per["pcd"])
            print(f"{name:22s} over {args.replicas} replicas: lvx {out[name]['lvx']['median_us']:8.1f} us ({lvx_reps})"
                  f"   pcd {out[name]['pcd']['median_us']:8.1f} us ({pcd_reps})", flush=True)
    print(json.dumps(out))
    if bad:
        raise SystemExit(f"outputs differ from {os.path.basename(libs[0])}: {bad}")


if __name__ == "__main__":
    main()
