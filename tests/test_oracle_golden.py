"""Pins the CPU oracle (oracle/) to golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest
from scipy.spatial.transform import Rotation, Slerp

from conftest import GOLDEN, golden, pkg
from oracle import restatement as R
from oracle import synth

SCEN = {"urban_complex": [0, 1, 2, 599, 1199], "parking_detailed": [0, 300], "highway_simple": [0, 1, 55]}
CFGS = {
    "urban_complex": {"duration": 120.0, "trajectory_type": "figure_eight",
                      "environment_complexity": "complex", "max_speed": 12.0, "lidar_fps": 10},
    "highway_simple": {"duration": 60.0, "trajectory_type": "linear",
                       "environment_complexity": "simple", "max_speed": 25.0, "lidar_fps": 15},
    "parking_detailed": {"duration": 30.0, "trajectory_type": "circular",
                         "environment_complexity": "medium", "max_speed": 5.0, "lidar_fps": 20},
}


def test_euler_matrix_matches_scipy_and_csim_builder():
    rng = np.random.default_rng(0)
    rpy = rng.uniform(-np.pi, np.pi, (200, 3))
    ours = R.euler_xyz_matrix(rpy)
    ref = Rotation.from_euler("xyz", rpy).as_matrix()
    np.testing.assert_allclose(ours, ref, atol=1e-14)
    # CSIM:187-212 explicit Rz @ Ry @ Rx
    for (r, p, y), M in zip(rpy[:20], ours[:20]):
        Rx = np.array([[1, 0, 0], [0, np.cos(r), -np.sin(r)], [0, np.sin(r), np.cos(r)]])
        Ry = np.array([[np.cos(p), 0, np.sin(p)], [0, 1, 0], [-np.sin(p), 0, np.cos(p)]])
        Rz = np.array([[np.cos(y), -np.sin(y), 0], [np.sin(y), np.cos(y), 0], [0, 0, 1]])
        np.testing.assert_allclose(M, Rz @ Ry @ Rx, atol=1e-15)
    q = R.euler_xyz_quat(rpy)
    np.testing.assert_allclose(np.abs(np.sum(q * Rotation.from_euler("xyz", rpy).as_quat(), axis=1)), 1.0,
                               atol=1e-13)


def test_transform_pointcloud_known_answers():
    g = golden("lmc_kat.npz")
    pts = g["points"]
    for i in range(int(g["n_cases"])):
        out = R.transform_pointcloud(pts, {"translation": g[f"t{i}"], "rotation": g[f"r{i}"]})
        np.testing.assert_allclose(out, g[f"out{i}"], rtol=0, atol=1e-12)
    # zero rotation => pure translation; yaw=pi/2 maps (x,y) -> (-y,x); intensity exact
    np.testing.assert_allclose(g["out1"][:, :3], pts[:, :3] + g["t1"], atol=1e-12)
    np.testing.assert_allclose(g["out2"][:, 0], -pts[:, 1], atol=1e-12)
    np.testing.assert_allclose(g["out2"][:, 1], pts[:, 0], atol=1e-12)
    assert np.array_equal(g["out3"][:, 3], pts[:, 3])
    assert g["empty_out"].shape == (0, 4)
    assert R.transform_pointcloud(np.zeros((0, 4)), {"translation": np.zeros(3), "rotation": np.zeros(3)}).shape == (0, 4)


@pytest.mark.parametrize("name", list(SCEN))
def test_frame_alignment_matches_reference(name):
    g = golden("lmc_frames.npz")
    tr = golden(f"lmc_traj_{name}.npz")
    times = pkg().trajectory.lidar_times(dict(pkg().default_config(), **CFGS[name]))
    assert len(times) == int(g[f"{name}/n_frames"])
    for fid in SCEN[name]:
        k = f"{name}/{fid}"
        assert float(times[fid]) == float(g[k + "/t_frame"])
        idx = int(R.select_pose_index(tr["time"], times[fid]))
        assert idx == int(g[k + "/pose_idx"]), (name, fid)
        out = R.align_frames([g[k + "/points_local"]], {"time": tr["time"], "position_gps": tr["position_gps"],
                                                         "orientation_imu": tr["orientation_imu"]}, [times[fid]])[0]
        np.testing.assert_allclose(out, g[k + "/aligned"], rtol=0, atol=1e-10)
    # the reference's empty frame stays (0,4)
    if name == "highway_simple":
        assert g["highway_simple/55/points_local"].shape == (0, 4)
        assert g["highway_simple/55/aligned"].shape == (0, 4)


@pytest.mark.parametrize("name", list(SCEN))
def test_product_pose_tables_bitwise_equal_reference(name):
    m = pkg()
    sim = m.LiDARMotionSimulator(dict(CFGS[name]))   # seeds np.random like LMC:288
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    ref = golden(f"lmc_traj_{name}.npz")
    for key in ("time", "position", "velocity", "orientation", "position_gps", "orientation_imu", "acceleration"):
        assert np.array_equal(tr[key], ref[key]), key


CASES = ["mid", "before", "after", "dup", "spike", "noimu"]


@pytest.mark.parametrize("case", CASES)
def test_pathb_vectorised_matches_reference(case):
    g = golden("csim_pathb.npz")
    out = R.compensate_arrays(g[f"{case}/xyz"], g[f"{case}/ts"], int(g[f"{case}/frame_start"]),
                              g[f"{case}/imu_ts"], g[f"{case}/imu_gyro"])
    np.testing.assert_allclose(out, g[f"{case}/out_xyz"], rtol=0, atol=1e-9)
    meta = g[f"{case}/out_meta"]
    assert np.array_equal(meta[:, 0], g[f"{case}/intensity"])
    assert np.array_equal(meta[:, 1], g[f"{case}/ts"])


@pytest.mark.parametrize("case", ["dup", "before", "after"])
def test_pathb_literal_loop_matches_reference(case):
    g = golden("csim_pathb.npz")
    imu = [(int(t), *gy, *ac) for t, gy, ac in zip(g[f"{case}/imu_ts"], g[f"{case}/imu_gyro"], g[f"{case}/imu_accel"])]
    sel = slice(0, 60)
    pts = [(x, y, z, int(i), int(t), 0, 0) for (x, y, z), i, t in
           zip(g[f"{case}/xyz"][sel], g[f"{case}/intensity"][sel], g[f"{case}/ts"][sel])]
    out = R.compensate_point_cloud_loop(pts, imu, int(g[f"{case}/frame_start"]))
    np.testing.assert_allclose(np.array([o[:3] for o in out]), g[f"{case}/out_xyz"][sel], rtol=0, atol=1e-12)


def test_pathb_duplicate_timestamp_semantics():
    g = golden("csim_pathb.npz")
    ts, gy = g["dup/imu_ts"], g["dup/imu_gyro"]
    dup_t = ts[np.flatnonzero(np.diff(ts) == 0)[0]]
    w = R.imu_interpolate_gyro(ts, gy, np.array([dup_t]))
    # at the duplicated time the later duplicate is 'before' (last sample with ts <= t)
    k = np.flatnonzero(ts == dup_t)[-1]
    np.testing.assert_allclose(w[0], gy[k], atol=0)


def test_slerp_matches_scipy_across_yaw_wrap():
    g = golden("slerp.npz")
    tr = {"time": g["time"], "position_gps": g["position_gps"], "orientation_imu": g["orientation_imu"]}
    Rm, p = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"], g["tq"])
    out = np.einsum("nij,nj->ni", Rm, g["xyz"]) + p
    np.testing.assert_allclose(out, g["out"], rtol=0, atol=1e-9)
    # at pose-sample times it reduces to Path A's transform with that sample
    for j in range(3):
        k = int(np.searchsorted(tr["time"], g["tq"][j]))
        ref = R.transform_pointcloud(np.column_stack([g["xyz"][j:j + 1], [0.0]]),
                                     {"translation": tr["position_gps"][k], "rotation": tr["orientation_imu"][k]})
        np.testing.assert_allclose(out[j], ref[0, :3], atol=1e-9)


def test_slerp_vs_scipy_random_and_clamped():
    rng = np.random.default_rng(3)
    T = 50
    time = np.linspace(0, 10, T)
    rpy = rng.uniform(-np.pi, np.pi, (T, 3))
    pos = rng.normal(0, 100, (T, 3))
    tq = rng.uniform(0, 10, 500)
    Rm, p = R.slerp_pose(time, pos, rpy, tq)
    ref = Slerp(time, Rotation.from_euler("xyz", rpy))(tq).as_matrix()
    np.testing.assert_allclose(Rm, ref, atol=1e-9)
    Rm2, p2 = R.slerp_pose(time, pos, rpy, np.array([-5.0, 20.0]))
    np.testing.assert_allclose(Rm2[0], R.euler_xyz_matrix(rpy[0]), atol=1e-12)
    np.testing.assert_allclose(p2[1], pos[-1], atol=1e-12)


def test_synth_generator_matches_committed_vectors():
    g = golden("synth.npz")
    x, y, z, i, t = synth.synth_frame(100_000, 0, 1000)
    for name, col in zip("xyzit", (x, y, z, i, t)):
        assert np.array_equal(col[:4096], g[name]), name
    sums = [c.astype(np.float64).sum() for c in (x, y, z, i, t)]
    np.testing.assert_allclose(sums, g["sums"], rtol=1e-12)
    # inside the Mid-70 FOV and range envelope
    assert (x >= 0.05).all() and (x < 90.0).all()
    assert (np.abs(np.degrees(np.arctan2(y, x))) <= 35.2 + 1e-4).all()
    el = np.degrees(np.arcsin(z / np.sqrt(x.astype(np.float64) ** 2 + y ** 2 + z ** 2)))
    assert (np.abs(el) <= 38.6 + 1e-4).all()
    assert t[0] == 0 and (np.diff(t) >= 0).all() and t[-1] < 100_000_000


def restore_rng(env_fixture):
    np.random.set_state(("MT19937", env_fixture["rng_keys"], int(env_fixture["rng_pos"]),
                         int(env_fixture["rng_has_gauss"]), float(env_fixture["rng_cached"])))


@pytest.mark.parametrize("name", list(SCEN))
def test_scan_environment_replays_reference_frame_loop(name):
    """LMC:802-832 replayed with the oracle's scan: every frame's point count and the recorded
    frames' local scans and aligned clouds match the reference run (same RNG stream)."""
    g = golden("lmc_frames.npz")
    e = golden(f"lmc_env_{name}.npz")
    tr = golden(f"lmc_traj_{name}.npz")
    m = pkg()
    cfg = dict(m.default_config(), **CFGS[name])
    times = m.trajectory.lidar_times(cfg)
    restore_rng(e)
    idx = R.select_pose_index(tr["time"], times)
    counts = []
    want = set(SCEN[name])
    for f, t in enumerate(times):
        pose = {"position": tr["position_gps"][idx[f]], "orientation": tr["orientation_imu"][idx[f]]}
        scan = R.scan_environment(e["environment"], pose, cfg)
        counts.append(len(scan))
        if f in want:
            np.testing.assert_allclose(scan, g[f"{name}/{f}/points_local"], rtol=0, atol=1e-9)
            al = R.transform_pointcloud(scan, {"translation": pose["position"], "rotation": pose["orientation"]})
            np.testing.assert_allclose(al, g[f"{name}/{f}/aligned"], rtol=0, atol=1e-9)
    assert np.array_equal(np.array(counts), g[f"{name}/frame_counts"])


def test_golden_files_are_data_only():
    for f in os.listdir(GOLDEN):
        assert f.endswith((".npz", ".json", ".py")), f
    with open(os.path.join(GOLDEN, "lmc_config.json")) as fh:
        json.load(fh)


def test_lvx_packer_bytes_match_reference():
    from oracle import codecs as C
    g = golden("codecs.npz")
    frames = [{"frame_id": int(g[f"lvx/{i}/frame_id"]), "timestamp": float(g[f"lvx/{i}/timestamp"]),
               "points": g[f"lvx/{i}/points"]} for i in range(int(g["lvx/n_frames"]))]
    assert C.lvx_bytes(frames) == g["lvx/bytes"].tobytes()
    pos = C.lvx_frame_positions([len(f["points"]) for f in frames])
    assert pos[-1] == len(g["lvx/bytes"])
    assert not bool(g["lvx/nan_ok"])
    with pytest.raises(ValueError):
        C.lvx_bytes([{"frame_id": 0, "timestamp": 0.0, "points": np.array([[np.nan, 0, 0, 0.5]])}])


@pytest.mark.parametrize("case", ["tricky", "specials", "random", "f32", "empty", "wide"])
def test_pcd_ascii_bytes_match_reference(case):
    from oracle import codecs as C
    g = golden("codecs.npz")
    assert C.pcd_ascii_bytes(g[f"pcd/{case}/points"]) == g[f"pcd/{case}/bytes"].tobytes()


def test_coordinate_transformer_matches_reference():
    g = golden("coords.npz")
    T = R.create_transform_matrix([10.0, -5.0, 2.0], [0.1, -0.2, 2.5])
    np.testing.assert_allclose(T, g["T/sensor/local"], atol=1e-14)
    np.testing.assert_allclose(np.linalg.inv(T), g["T/local/sensor"], atol=1e-12)
    np.testing.assert_allclose(R.transform_points_h(g["p3"], T), g["tp/sensor/local"], atol=1e-12)
    np.testing.assert_allclose(R.transform_points_h(g["p3"], np.linalg.inv(T)), g["tp/local/sensor"], atol=1e-12)
    np.testing.assert_allclose(R.transform_points_h(g["p4"], T), g["tp4/sensor/local"], atol=1e-12)
    Tsv = np.eye(4)
    Tsv[2, 3] = 1.5
    np.testing.assert_allclose(R.transform_points_h(g["p3"], Tsv), g["tp/sensor/vehicle"], atol=1e-12)
    assert np.array_equal(g["tp/vehicle/sensor"], g["p3"])          # missing pair: input unchanged
    for i in range(int(g["tc/n_frames"])):
        assert np.array_equal(g[f"tc/utm/{i}"], g[f"tc/in/{i}"])    # utm package absent: unchanged
