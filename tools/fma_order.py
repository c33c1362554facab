"""Which accumulation order numpy's matmul uses for the reference's 3x3 (and 4x4) transforms.

The float64 row kernels (kernels.hpp frame_apply / k_affine_rows_f64, scan.hpp scan_rotate) repeat
it so that their outputs equal the reference's values bit for bit.  Compiles a tiny C helper with
gcc into a temp dir and compares, on random data, numpy's

    (R.T @ d.T).T         LMC:728   (scan_environment)
    (R @ p.T).T + t       LMC:775   (transform_pointcloud)
    (T @ [p, w].T).T      CSIM:230  (CoordinateTransformer.transform_points)

with three candidate orders per output: plain left-to-right sums, the ascending FMA chain
fma(a2, x2, fma(a1, x1, a0 * x0)) and the descending one.  Measured in the build container
(OpenBLAS 0.3.29 Haswell-family dgemm, the box the golden fixtures come from): the ascending chain
matches every value, the others miss 25-45 %.

One-row products (a frame of one point; CSIM:2137's per-point transform_points) go through dgemv
and sum in other orders, checked here as "single": 3x3 fma(a2, x2, fma(a0, x0, a1 * x1)), 4x4
(a0 x0 + a2 x2) + (a1 x1 + a3 x3) with every product rounded (frame_apply(single) and
k_affine_rows_f64's per-row order).  Row counts 2..257 and 1000 all take the ascending chain.
The exception is LMC:728 with one scene point in range: R.T is F-contiguous there, and its
(3,3) @ (3,1) product keeps the ascending chain (0 of 60 000 values differ; "single" misses 23 %),
so scan.hpp's scan_rotate needs no one-point order (round 6).

    python tools/fma_order.py
"""
import ctypes
import os
import subprocess
import tempfile

import numpy as np
from scipy.spatial.transform import Rotation

C_SRC = r"""
#include <math.h>
#include <stdint.h>
void chain(const double* A, int K, const double* X, int64_t n, int order, double* o) {
  for (int64_t r = 0; r < n; ++r)
    for (int i = 0; i < 3; ++i) {
      const double* a = A + K * i; const double* x = X + K * r; double s;
      if (order == 0) { s = a[0] * x[0]; for (int k = 1; k < K; ++k) s = s + a[k] * x[k]; }
      else if (order == 1) { s = a[0] * x[0]; for (int k = 1; k < K; ++k) s = fma(a[k], x[k], s); }
      else if (order == 2) { s = a[K - 1] * x[K - 1]; for (int k = K - 2; k >= 0; --k) s = fma(a[k], x[k], s); }
      else if (K == 3) s = fma(a[2], x[2], fma(a[0], x[0], a[1] * x[1]));            /* one-row 3x3 */
      else s = (a[0] * x[0] + a[2] * x[2]) + (a[1] * x[1] + a[3] * x[3]);           /* one-row 4x4 */
      o[3 * r + i] = s;
    }
}
"""


def main():
    d = tempfile.mkdtemp()
    src, so = os.path.join(d, "c.c"), os.path.join(d, "c.so")
    open(src, "w").write(C_SRC)
    subprocess.run(["gcc", "-O2", "-mfma", "-ffp-contract=off", "-shared", "-fPIC", src, "-o", so, "-lm"], check=True)
    lib = ctypes.CDLL(so)

    def run(A, X, order):
        A = np.ascontiguousarray(A)
        X = np.ascontiguousarray(X)
        o = np.empty((len(X), 3))
        lib.chain(ctypes.c_void_p(A.ctypes.data), ctypes.c_int(A.shape[1]), ctypes.c_void_p(X.ctypes.data),
                  ctypes.c_int64(len(X)), ctypes.c_int(order), ctypes.c_void_p(o.ctypes.data))
        return o

    rng = np.random.default_rng(0)
    n = 200_000
    R = Rotation.from_euler("xyz", rng.uniform(-3, 3, 3)).as_matrix()
    t = rng.normal(0, 30, 3)
    d3 = rng.uniform(-100, 100, (n, 3))
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = [5e5, 4.43e6, 3.0]
    p4 = np.column_stack([d3, rng.uniform(0, 1, n)])
    cases = {
        "LMC:728 (R.T @ d.T).T": ((R.T @ d3.T).T, R.T, d3, None),
        "LMC:775 (R @ p.T).T + t": ((R @ d3.T).T + t, R, d3, t),
        "CSIM:230 T @ [p, 1]": ((T @ np.column_stack([d3, np.ones(n)]).T).T[:, :3], T[:3], np.column_stack([d3, np.ones(n)]), None),
        "CSIM:230 T @ [p, w]": ((T @ p4.T).T[:, :3], T[:3], p4, None),
    }
    for name, (ref, A, X, add) in cases.items():
        miss = []
        for order in range(3):
            o = run(A, X, order)
            if add is not None:
                o = o + add
            miss.append(int(np.count_nonzero(o != ref)))
        print(f"{name:28s} values {ref.size}: mismatches plain {miss[0]}, fma ascending {miss[1]}, "
              f"fma descending {miss[2]}")

    # one-row products, one numpy call per point (dgemv): the "single" order (order 3)
    m = 20_000
    single = {"LMC:775 one point (R @ p.T).T + t": [], "CSIM:230 one point T @ [p, w]": [],
              "LMC:728 one point (R.T @ d.T).T": []}
    miss = {k: [0, 0] for k in single}
    for i in range(m):
        p = d3[i:i + 1]
        for name, ref, A, X, add in (
                ("LMC:775 one point (R @ p.T).T + t", (R @ p.T).T + t, R, p, t),
                ("CSIM:230 one point T @ [p, w]", (T @ p4[i:i + 1].T).T[:, :3], T[:3], p4[i:i + 1], None),
                # scan_environment with one scene point in range: R.T is F-contiguous here
                ("LMC:728 one point (R.T @ d.T).T", (R.T @ p.T).T, R.T, p, None)):
            for j, order in enumerate((1, 3)):
                o = run(A, X, order)
                if add is not None:
                    o = o + add
                miss[name][j] += int(np.count_nonzero(o != ref))
    for name, (asc, one) in miss.items():
        print(f"{name:34s} values {3 * m}: mismatches fma ascending {asc}, single {one}")
    # several rows: the ascending chain at every small count
    small = [k for k in list(range(2, 70)) + [255, 256, 257, 1000]
             if not np.array_equal(run(R, d3[:k], 1) + t, (R @ d3[:k].T).T + t)]
    print("row counts 2..69, 255-257, 1000 not matching the ascending chain:", small)


if __name__ == "__main__":
    main()
