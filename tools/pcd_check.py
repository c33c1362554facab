"""Check the device PCD encoder of one or more library builds against the oracle on the bench's
synthetic frames (f64 AoS device source, as tools/ab_codecs.py encodes).  GPU box only.

    python tools/pcd_check.py --libs build/variants/lib_packed.so,build/variants/lib_bytes.so
"""
import argparse
import os
import sys
from ctypes import c_int64

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mcamd as mc  # noqa: E402
from oracle import codecs as C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--points", type=int, default=100_000)
    args = ap.parse_args()
    counts = np.full(args.frames, args.points, np.int64)
    F = len(counts)
    bad = 0
    for lib in args.libs.split(","):
        ctx = mc.Context(0, lib_path=lib)
        b = ctx.batch(counts)
        b.synth(seed=0, frame_id_base=1000)
        host = b.split(b.download_aos())
        src = ctx.device_buffer(int(counts.sum()) * 32)
        b.fetch_aos_device(src)
        cap = int(counts.sum()) * 48
        out = ctx.device_buffer(cap)
        bpos = np.zeros(F + 1, np.int64)
        mc._lib.check(ctx.lib.mc_pcd_encode(ctx.handle, src.ptr, 4, F, mc._lib.ptr(counts, c_int64), out.ptr, cap,
                                            mc._lib.ptr(bpos, c_int64)), "pcd_encode")
        text = np.empty(int(bpos[-1]), np.uint8)
        mc._lib.check(ctx.lib.mc_memcpy_d2h(ctx.handle, text.ctypes.data, out.ptr.value, text.size), "d2h")
        for f in range(F):
            want = C.pcd_ascii_bytes(host[f])
            want = want[want.index(b"DATA ascii\n") + 11:]
            got = text[bpos[f]:bpos[f + 1]].tobytes()
            if got != want:
                bad += 1
                i = next((k for k in range(min(len(got), len(want))) if got[k] != want[k]), min(len(got), len(want)))
                g_ = np.frombuffer(got, np.uint8)
                w_ = np.frombuffer(want, np.uint8)
                nd = int((g_ != w_).sum()) if len(g_) == len(w_) else -1
                line = want[:i].count(b"\n")
                print(f"{os.path.basename(lib)} frame {f}: MISMATCH at byte {i} (line {line}, tile {line // 256}, "
                      f"lane {line % 256}; {nd} bytes differ; len {len(got)} vs {len(want)}): "
                      f"got {got[max(0, i - 60):i + 60]!r} want {want[max(0, i - 60):i + 60]!r}", flush=True)
                if bad > 6:
                    break
        print(f"{os.path.basename(lib)}: done, {bad} bad frames so far", flush=True)
        out.close()
        src.close()
        b.close()
        ctx.close()
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
