"""The opt-in latency server (mc_set_latency_server, k_lat_server): single transform_pointcloud calls
(LMC:772-776, one frame per call as LMC:831 makes them) served by a resident workgroup polling a
mailbox in pinned host memory — results equal the launched kernel's, the oracle's at the strict bar,
for any row count up to 32768 and row width >= 4; it relaunches itself after its idle exit, and
disabling it / closing the context with it running returns (bounded exits)."""
import time

import numpy as np
import pytest

from conftest import assert_scaled_close
from oracle import restatement as R

pytestmark = pytest.mark.gpu


def test_latency_server_matches_kernel_and_oracle(mc, gpu_ctx):
    sim = mc.LiDARMotionSimulator(context=gpu_ctx)
    rng = np.random.default_rng(3)
    cases = []
    for n in (1, 7, 255, 1600, 4097, 32768):
        for ld in (4, 6):
            pts = np.column_stack([rng.normal(0, 40, (n, 3)), rng.uniform(0, 1, (n, ld - 3))])
            pose = {"translation": rng.normal(0, 50, 3), "rotation": rng.uniform(-3.1, 3.1, 3)}
            cases.append((pts, pose, sim.transform_pointcloud(pts, pose)))
    info = gpu_ctx.latency_server(True)
    try:
        assert info["enabled"]
        for rep in range(3):
            for pts, pose, base in cases:
                got = sim.transform_pointcloud(pts, pose)
                assert got.shape == (len(pts), 4)
                assert np.array_equal(got[:, 3], pts[:, 3])
                ref = R.transform_pointcloud(pts, pose)
                scale = np.linalg.norm(pts[:, :3], axis=1) + np.linalg.norm(pose["translation"])
                assert_scaled_close(got[:, :3], ref[:, :3], scale, what=f"n={len(pts)}")
                assert np.allclose(got, base, rtol=0, atol=1e-12 * (1 + np.abs(base)).max())
        served = gpu_ctx.latency_server_info()
        assert served["requests"] == 3 * len(cases)
        time.sleep(0.2)                     # past the server's idle exit: the next call relaunches it
        pts, pose, base = cases[3]
        assert np.allclose(sim.transform_pointcloud(pts, pose), base, rtol=0, atol=1e-9)
        assert gpu_ctx.latency_server_info()["launches"] >= served["launches"] + 1
        big = np.column_stack([rng.normal(0, 40, (40_000, 3)), np.zeros(40_000)])   # above the server's range
        ref = R.transform_pointcloud(big, pose)
        got = sim.transform_pointcloud(big, pose)
        assert_scaled_close(got[:, :3], ref[:, :3], np.linalg.norm(big[:, :3], axis=1) + np.linalg.norm(pose["translation"]))
    finally:
        assert not gpu_ctx.latency_server(False)["enabled"]


def test_latency_server_closed_with_context(mc):
    ctx = mc.Context(0)
    ctx.latency_server(True)
    sim = mc.LiDARMotionSimulator(context=ctx)
    pts = np.column_stack([np.ones((100, 3)), np.zeros(100)])
    out = sim.transform_pointcloud(pts, {"translation": np.zeros(3), "rotation": np.zeros(3)})
    assert np.array_equal(out, pts)
    t0 = time.perf_counter()
    ctx.close()                            # quit flag -> the resident workgroup returns
    assert time.perf_counter() - t0 < 5.0
