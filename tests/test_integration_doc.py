"""The ctypes stub that INTEGRATION.md tells a maintainer to paste into the reference must work
as written: run it against the built library and compare with the oracle."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, assert_scaled_close, golden, scale_of
from oracle import restatement as R


def _stub_source():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        blocks = re.findall(r"```python\n(.*?)```", f.read(), flags=re.S)
    src = [b for b in blocks if "def transform_pointcloud" in b]
    assert len(src) == 1
    lib = os.path.join(ROOT, "livox-motion-compensation-sim_amd", "libmcdeskew.so")
    return src[0].replace("/path/to/livox-motion-compensation-sim_amd/libmcdeskew.so", lib)


def test_stub_compiles():
    compile(_stub_source(), "INTEGRATION.md", "exec")


@pytest.mark.gpu
def test_stub_matches_reference_known_answers():
    ns = {}
    exec(compile(_stub_source(), "INTEGRATION.md", "exec"), ns)
    g = golden("lmc_kat.npz")
    pts = g["points"]
    for i in range(int(g["n_cases"])):
        out = ns["transform_pointcloud"](None, pts, {"translation": g[f"t{i}"], "rotation": g[f"r{i}"]})
        assert out.shape == (len(pts), 4) and out.dtype == np.float64
        assert_scaled_close(out[:, :3], g[f"out{i}"][:, :3], scale_of(pts[:, :3], g[f"t{i}"]))
        assert np.array_equal(out, g[f"out{i}"])   # the reference's float64 values, bit for bit
    assert ns["transform_pointcloud"](None, np.zeros((0, 4)), {"translation": np.zeros(3),
                                                              "rotation": np.zeros(3)}).shape == (0, 4)
    with pytest.raises(IndexError):
        ns["transform_pointcloud"](None, np.zeros((3, 3)), {"translation": np.zeros(3), "rotation": np.zeros(3)})
    ref = R.transform_pointcloud(pts, {"translation": g["t3"], "rotation": g["r3"]})
    np.testing.assert_allclose(ns["transform_pointcloud"](None, pts, {"translation": g["t3"], "rotation": g["r3"]})[:, 3],
                               ref[:, 3], rtol=1e-7)


def _pcd_stub_source():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        blocks = re.findall(r"```python\n(.*?)```", f.read(), flags=re.S)
    src = [b for b in blocks if "def save_pcd" in b]
    assert len(src) == 1
    lib = os.path.join(ROOT, "livox-motion-compensation-sim_amd", "libmcdeskew.so")
    return src[0].replace("/path/to/livox-motion-compensation-sim_amd/libmcdeskew.so", lib)


def test_pcd_stub_compiles():
    compile(_pcd_stub_source(), "INTEGRATION.md", "exec")


@pytest.mark.gpu
def test_pcd_stub_writes_reference_bytes(tmp_path):
    ns = {}
    exec(compile(_pcd_stub_source(), "INTEGRATION.md", "exec"), ns)
    g = golden("codecs.npz")
    for case in ("tricky", "specials", "random", "empty", "wide"):
        fn = str(tmp_path / f"{case}.pcd")
        ns["save_pcd"](None, g[f"pcd/{case}/points"], fn)
        with open(fn, "rb") as f:
            assert f.read() == g[f"pcd/{case}/bytes"].tobytes(), case


def _pathb_stub_source():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        blocks = re.findall(r"```python\n(.*?)```", f.read(), flags=re.S)
    src = [b for b in blocks if "def compensate_point_cloud" in b]
    assert len(src) == 1
    lib = os.path.join(ROOT, "livox-motion-compensation-sim_amd", "libmcdeskew.so")
    return src[0].replace("/path/to/livox-motion-compensation-sim_amd/libmcdeskew.so", lib)


def test_pathb_stub_compiles():
    compile(_pathb_stub_source(), "INTEGRATION.md", "exec")


@pytest.mark.gpu
def test_pathb_stub_matches_reference_goldens(mc):
    """The stub a maintainer pastes over CSIM:1435-1480, run on the reference's own golden cases:
    strict parity with the reference's float64 output, metadata and pass-through rules kept."""
    ns = {}
    exec(compile(_pathb_stub_source(), "INTEGRATION.md", "exec"), ns)
    g = golden("csim_pathb.npz")

    class Comp:
        enable_compensation = True
    for case in ("mid", "before", "after", "dup", "spike", "noimu"):
        imu = [mc.IMUData(int(t), *map(float, gy), *map(float, ac))
               for t, gy, ac in zip(g[f"{case}/imu_ts"], g[f"{case}/imu_gyro"], g[f"{case}/imu_accel"])]
        xyz = g[f"{case}/xyz"]
        pts = [mc.LiDARPoint(float(p[0]), float(p[1]), float(p[2]), int(i), int(t), int(r), int(tg))
               for p, i, t, r, tg in zip(xyz, g[f"{case}/intensity"], g[f"{case}/ts"], g[f"{case}/ring"],
                                         g[f"{case}/tag"])]
        out = ns["compensate_point_cloud"](Comp(), pts, imu, int(g[f"{case}/frame_start"]), 100_000_000)
        if case == "noimu":
            assert out is pts
            continue
        got = np.array([[p.x, p.y, p.z] for p in out])
        assert_scaled_close(got, g[f"{case}/out_xyz"], scale_of(xyz), what=case)
        meta = np.array([[p.intensity, p.timestamp, p.ring, p.tag] for p in out])
        assert np.array_equal(meta, g[f"{case}/out_meta"])
