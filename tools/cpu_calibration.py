"""Time the reference itself next to the oracle restatement, in the build container.

The GPU box has no /root/reference, so bench.py's cpu_baseline times the oracle (oracle/) on the
box's cores; this script shows how that CPU leg relates to the real reference code on the same
inputs and the same core (one BLAS thread).  Run here only:

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_calibration.py   ->  profiles/cpu_calibration.json
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys
import tempfile
import time

import numpy as np
from threadpoolctl import threadpool_limits

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from make_golden import import_reference  # noqa: E402
from oracle import codecs as C  # noqa: E402
from oracle import restatement as R  # noqa: E402
from oracle import synth  # noqa: E402


def best(fn, reps=5):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    lmc, csim = import_reference()
    out = {"host": os.uname().nodename, "cores_available": len(os.sched_getaffinity(0)), "threads": 1}
    x, y, z, i, t = synth.synth_frame(100_000, 0, 1000)
    pts = np.column_stack([x, y, z, i]).astype(np.float64)
    pose = {"translation": np.array([12.0, -3.0, 0.5]), "rotation": np.array([0.01, -0.02, 1.3])}
    with threadpool_limits(limits=1), contextlib.redirect_stdout(io.StringIO()):
        sim = lmc.LiDARMotionSimulator()
        ref = best(lambda: sim.transform_pointcloud(pts, pose))
        ora = best(lambda: R.transform_pointcloud(pts, pose))
        out["transform_pointcloud_100k"] = {"reference_s": ref, "oracle_s": ora, "oracle_over_reference": ref / ora,
                                            "reference_Mpts_s": 1e5 / ref / 1e6, "oracle_Mpts_s": 1e5 / ora / 1e6}

        # Path B: the reference's per-point Python loop vs the vectorised oracle
        n = 2000
        ts = (np.arange(n) * (100_000_000 // n)).astype(np.int64)
        imu_ts = np.arange(0, 200_000_000, 5_000_000, dtype=np.int64)
        gyro = np.column_stack([0.1 * np.sin(imu_ts * 1e-8), 0.05 * np.ones(len(imu_ts)), 0.3 * np.cos(imu_ts * 1e-8)])
        imu = [csim.IMUData(int(a), *map(float, g), 0.0, 0.0, 9.81) for a, g in zip(imu_ts, gyro)]
        lp = [csim.LiDARPoint(float(a), float(b), float(c), 10, int(s), 0, 0) for (a, b, c), s in zip(pts[:n, :3], ts)]
        mcomp = csim.MotionCompensator(dict(csim.DEFAULT_CONFIG))
        ref = best(lambda: mcomp.compensate_point_cloud(lp, imu, 0, 100_000_000), reps=2)
        ora = best(lambda: R.compensate_arrays(pts[:n, :3], ts, 0, imu_ts, gyro))
        out["compensate_point_cloud_2k"] = {"reference_s": ref, "oracle_s": ora, "oracle_over_reference": ref / ora,
                                            "reference_Mpts_s": n / ref / 1e6, "oracle_Mpts_s": n / ora / 1e6}

        # scan_environment on the reference's own urban scene
        g = np.load(os.path.join(ROOT, "tests", "golden", "lmc_env_urban_complex.npz"))
        env = g["environment"]
        spose = {"position": np.array([5.0, 2.0, 1.8]), "orientation": np.array([0.0, 0.01, 0.7])}
        cfg = dict(sim.config)
        ref = best(lambda: sim.scan_environment(env, spose))
        ora = best(lambda: R.scan_environment(env, spose, cfg))
        out["scan_environment_29k_scene"] = {"reference_s": ref, "oracle_s": ora, "oracle_over_reference": ref / ora}

        # writers
        frames = [{"frame_id": 0, "timestamp": 0.0, "points": pts[:20_000]}]
        w = lmc.LivoxLVXWriter()
        with tempfile.TemporaryDirectory() as d:
            ref = best(lambda: w.write_compatible_lvx(os.path.join(d, "a.lvx"), frames), reps=2)
            ora = best(lambda: C.lvx_bytes(frames))
            out["lvx_20k"] = {"reference_s": ref, "oracle_s": ora, "oracle_over_reference": ref / ora,
                              "reference_Mpts_s": 2e4 / ref / 1e6, "oracle_Mpts_s": 2e4 / ora / 1e6}
            ref = best(lambda: sim.save_pcd(pts[:20_000], os.path.join(d, "a.pcd")), reps=2)
            ora = best(lambda: C.pcd_ascii_bytes(pts[:20_000]), reps=2)
            out["pcd_20k"] = {"reference_s": ref, "oracle_s": ora, "oracle_over_reference": ref / ora,
                              "reference_Mpts_s": 2e4 / ref / 1e6, "oracle_Mpts_s": 2e4 / ora / 1e6}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
