"""Host-side transfer ceilings on the GPU box (diagnostic): single-thread host memcpy, pinned
H2D / D2H DMA, pageable H2D / D2H through the HIP runtime, and pinned H2D + D2H at once on two
streams (the aggregate both directions carry together).  These bound the host-array entry
points (transform_pointcloud / run_alignment on numpy arrays), not the device-resident hot path.

    python tools/pcie_probe.py [--mb 256]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import time

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=256)
    args = ap.parse_args()
    nb = args.mb << 20
    hip = ctypes.CDLL("libamdhip64.so")
    out = {"bytes": nb}
    a = np.ones(nb // 8)
    b = np.empty_like(a)
    np.copyto(b, a)
    t0 = time.perf_counter()
    for _ in range(5):
        np.copyto(b, a)
    out["host_memcpy_GBs_1thread"] = 5 * nb / (time.perf_counter() - t0) / 1e9
    pin = ctypes.c_void_p()
    dev = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(pin), ctypes.c_size_t(nb), 0) == 0
    assert hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(nb)) == 0
    H2D, D2H = 1, 2
    for name, dst, src, kind in (("pinned_H2D", dev, pin, H2D), ("pinned_D2H", pin, dev, D2H),
                                 ("pageable_H2D", dev, ctypes.c_void_p(a.ctypes.data), H2D),
                                 ("pageable_D2H", ctypes.c_void_p(b.ctypes.data), dev, D2H)):
        assert hip.hipMemcpy(dst, src, ctypes.c_size_t(nb), kind) == 0
        hip.hipDeviceSynchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            hip.hipMemcpy(dst, src, ctypes.c_size_t(nb), kind)
        hip.hipDeviceSynchronize()
        out[name + "_GBs"] = 5 * nb / (time.perf_counter() - t0) / 1e9
    # both directions at once: H2D and D2H of nb bytes each on two streams (distinct buffers)
    pin2, dev2 = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(pin2), ctypes.c_size_t(nb), 0) == 0
    assert hip.hipMalloc(ctypes.byref(dev2), ctypes.c_size_t(nb)) == 0
    s1, s2 = ctypes.c_void_p(), ctypes.c_void_p()
    hip.hipStreamCreate(ctypes.byref(s1))
    hip.hipStreamCreate(ctypes.byref(s2))
    for rep in range(6):
        t0 = time.perf_counter()
        hip.hipMemcpyAsync(dev, pin, ctypes.c_size_t(nb), H2D, s1)
        hip.hipMemcpyAsync(pin2, dev2, ctypes.c_size_t(nb), D2H, s2)
        hip.hipStreamSynchronize(s1)
        hip.hipStreamSynchronize(s2)
        dt = time.perf_counter() - t0
        if rep:   # (the first pair warms up)
            out.setdefault("duplex_aggregate_GBs", []).append(2 * nb / dt / 1e9)
    hip.hipStreamDestroy(s1)
    hip.hipStreamDestroy(s2)
    hip.hipFree(dev2)
    hip.hipHostFree(pin2)
    hip.hipFree(dev)
    hip.hipHostFree(pin)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
