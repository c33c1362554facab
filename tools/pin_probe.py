"""Cost of pinning host memory on the GPU box (diagnostic for the host-array drop-in's output):
hipHostMalloc / hipHostFree of a config-2-sized (600 x 100k x 32 B) block, hipHostRegister of a
numpy array of that size, and pinned D2H into it.

    python tools/pin_probe.py [--gb 1.92]
"""
import argparse
import ctypes
import json
import time

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=1.92)
    args = ap.parse_args()
    nb = int(args.gb * 1e9)
    hip = ctypes.CDLL("libamdhip64.so")
    out = {"bytes": nb}
    dev = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(nb)) == 0
    for rep in range(2):
        p = ctypes.c_void_p()
        t0 = time.perf_counter()
        assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(nb), 0) == 0
        t1 = time.perf_counter()
        assert hip.hipMemcpy(p, dev, ctypes.c_size_t(nb), 2) == 0
        t2 = time.perf_counter()
        assert hip.hipHostFree(p) == 0
        t3 = time.perf_counter()
        out[f"hostmalloc_s_{rep}"] = t1 - t0
        out[f"d2h_into_it_s_{rep}"] = t2 - t1
        out[f"hostfree_s_{rep}"] = t3 - t2
    a = np.empty(nb // 8)
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(a.nbytes), 0)
    t1 = time.perf_counter()
    out["register_rc"] = rc
    out["register_fresh_s"] = t1 - t0
    if rc == 0:
        t0 = time.perf_counter()
        hip.hipMemcpy(ctypes.c_void_p(a.ctypes.data), dev, ctypes.c_size_t(a.nbytes), 2)
        out["d2h_into_registered_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data))
        out["unregister_s"] = time.perf_counter() - t0
    b = np.ones(nb // 8)
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(ctypes.c_void_p(b.ctypes.data), ctypes.c_size_t(b.nbytes), 0)
    out["register_touched_s"] = time.perf_counter() - t0
    if rc == 0:
        hip.hipHostUnregister(ctypes.c_void_p(b.ctypes.data))
    hip.hipFree(dev)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
