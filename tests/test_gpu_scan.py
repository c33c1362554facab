"""GPU parity of scan_environment (LMC:701-770) and of the fused scan -> align
frame loop (LMC:802-832) against the reference's own recorded runs (tests/golden/lmc_env_*.npz:
the scene and numpy's RNG state before the frame loop; lmc_frames.npz: every frame's point count
and the local / aligned clouds of selected frames) and against the oracle on synthetic scenes.

simulate_frames writes the reference's float64 arrays (mc_scan_emit_f64): counts, kept point sets
and every coordinate are compared bit for bit with the reference's run.  The float32 batch path
(scan_frames, the hot path's input layout) is held to the strict per-coordinate 1e-5.
"""
import numpy as np
import pytest

from conftest import assert_scaled_close, golden, scale_of
from oracle import restatement as R

pytestmark = pytest.mark.gpu

CFGS = {
    "urban_complex": {"duration": 120.0, "trajectory_type": "figure_eight",
                      "environment_complexity": "complex", "max_speed": 12.0, "lidar_fps": 10},
    "highway_simple": {"duration": 60.0, "trajectory_type": "linear",
                       "environment_complexity": "simple", "max_speed": 25.0, "lidar_fps": 15},
    "parking_detailed": {"duration": 30.0, "trajectory_type": "circular",
                         "environment_complexity": "medium", "max_speed": 5.0, "lidar_fps": 20},
}
SCEN = {"urban_complex": [0, 1, 2, 599, 1199], "parking_detailed": [0, 300], "highway_simple": [0, 1, 55]}


def restore_rng(e):
    np.random.set_state(("MT19937", e["rng_keys"], int(e["rng_pos"]), int(e["rng_has_gauss"]),
                         float(e["rng_cached"])))


def traj_of(name):
    g = golden(f"lmc_traj_{name}.npz")
    return {k: g[k] for k in g.files}


@pytest.mark.parametrize("name", list(SCEN))
def test_frame_loop_reproduces_reference_run(mc, gpu_ctx, name):
    g = golden("lmc_frames.npz")
    e = golden(f"lmc_env_{name}.npz")
    tr = traj_of(name)
    sim = mc.LiDARMotionSimulator(dict(CFGS[name]), context=gpu_ctx)
    times = sim.lidar_times()
    restore_rng(e)
    res = sim.simulate_frames(e["environment"], tr, times)
    counts = np.array([len(s["points_local"]) for s in res["raw_scans"]])
    assert np.array_equal(counts, g[f"{name}/frame_counts"])
    for f in SCEN[name]:
        k = f"{name}/{f}"
        loc = res["raw_scans"][f]["points_local"]
        al = res["aligned_pointclouds"][f]
        assert loc.dtype == np.float64 and al.dtype == np.float64
        # bit for bit: scipy's R (rot.cpp), numpy's matmul accumulation, the same noise draws
        assert np.array_equal(loc, g[k + "/points_local"]), (k, int(np.count_nonzero(loc != g[k + "/points_local"])))
        assert np.array_equal(al, g[k + "/aligned"]), (k, int(np.count_nonzero(al != g[k + "/aligned"])))
        pose = res["raw_scans"][f]["sensor_pose"]
        assert np.array_equal(pose["position"], g[k + "/position"]) and np.array_equal(pose["orientation"], g[k + "/rpy"])
        ref = R.transform_pointcloud(loc, {"translation": pose["position"], "rotation": pose["orientation"]})
        assert_scaled_close(al, ref, scale_of(loc[:, :3], pose["position"]), what=k + " aligned vs oracle")
    # the global RNG advanced by exactly the reference's draws: the next number matches a replay
    nxt = np.random.random()
    restore_rng(e)
    np.random.normal(0, 1, (int(counts.sum()), 3))
    assert np.random.random() == nxt
    assert len(res["motion_data"]) == len(times) and res["motion_data"][7]["frame_id"] == 7


def synth_scene(seed, n):
    rng = np.random.default_rng(seed)
    env = np.empty((n, 5))
    env[:, 0] = rng.uniform(-120, 120, n)
    env[:, 1] = rng.uniform(-120, 120, n)
    env[:, 2] = rng.uniform(-10, 25, n)
    env[:, 3] = rng.uniform(0, 1, n)
    env[:, 4] = 7.0   # extra column, ignored like the reference's environment[:, :3] / [:, 3]
    return env


@pytest.mark.parametrize("cap", [100_000, 257, 1])
def test_scan_noise_free_vs_oracle_random_poses(mc, gpu_ctx, cap):
    cfg = dict(range_max=90.0, range_min=0.5, fov_horizontal=70.4, fov_vertical=77.2,
               points_per_frame=cap, lidar_range_noise=0.0)
    sim = mc.LiDARMotionSimulator(cfg, context=gpu_ctx)
    env = synth_scene(5, 300_001)
    rng = np.random.default_rng(9)
    for _ in range(6):
        pose = {"position": rng.uniform(-40, 40, 3), "orientation": rng.uniform(-np.pi, np.pi, 3)}
        ref = R.scan_environment(env, pose, sim.config)
        out = sim.scan_environment(env, pose)
        assert out.shape == ref.shape
        assert_scaled_close(out, ref, scale_of(ref[:, :3]) + 1e-3, what=f"cap {cap}")
        assert out.dtype == np.float64 and np.array_equal(out[:, 3], ref[:, 3])


def test_scan_batched_frames_searchsorted_vs_oracle(mc, gpu_ctx):
    cfg = dict(points_per_frame=5000, lidar_range_noise=0.0)
    sim = mc.LiDARMotionSimulator(cfg, context=gpu_ctx)
    tr = traj_of("urban_complex")
    env = synth_scene(11, 200_000)
    env[:, :2] += tr["position_gps"][0, :2]
    times = np.linspace(0, 120, 37)
    b = sim.scan_frames(env, tr, times)
    got = b.split(b.download_aos())
    idx = R.select_pose_index(tr["time"], times)
    for f, k in enumerate(idx):
        ref = R.scan_environment(env, {"position": tr["position_gps"][k], "orientation": tr["orientation_imu"][k]},
                                 sim.config)
        assert got[f].shape == ref.shape, f
        assert_scaled_close(got[f], ref, scale_of(ref[:, :3]) + 1e-3, what=f"frame {f}")


def test_scan_edge_cases(mc, gpu_ctx):
    sim = mc.LiDARMotionSimulator({"lidar_range_noise": 0.0}, context=gpu_ctx)
    pose = {"position": np.zeros(3), "orientation": np.zeros(3)}
    # empty scene, everything out of range, everything behind the sensor
    assert sim.scan_environment(np.zeros((0, 4)), pose).shape == (0, 4)
    far = np.array([[1000.0, 0, 0, 0.5], [0, 2000.0, 0, 0.1]])
    assert sim.scan_environment(far, pose).shape == (0, 4)
    behind = np.array([[-10.0, 0, 0, 0.5], [-5.0, 1, 0, 0.5]])
    assert sim.scan_environment(behind, pose).shape == (0, 4)
    # a point on the sensor: range 0 < range_min; FOV edge exactly at fov/2
    edge = np.array([[0.0, 0, 0, 0.2], [10.0, 10.0 * np.tan(np.radians(10.0)), 0, 0.3], [10.0, 0, 0, 0.9]])
    ref = R.scan_environment(edge, pose, sim.config)
    out = sim.scan_environment(edge, pose)
    assert out.shape == ref.shape
    assert_scaled_close(out, ref, scale_of(ref[:, :3]), what="edge")
    # fewer than 4 columns: the reference fails indexing environment[:, 3] / [:, :3]
    with pytest.raises(IndexError):
        sim.scan_environment(np.zeros((5, 3)), pose)


def test_scan_fov_edges_decided_like_reference(mc, gpu_ctx):
    """Points at +-1e-12 .. 1e-3 degrees from the FOV edges: the kernel's transcendental-free test
    must defer to the reference's atan2 / asin comparisons near the edges (LMC:735-745)."""
    cfg = dict(lidar_range_noise=0.0, points_per_frame=10 ** 6)
    sim = mc.LiDARMotionSimulator(cfg, context=gpu_ctx)
    h, v = sim.config["fov_horizontal"] / 2, sim.config["fov_vertical"] / 2
    offs = np.concatenate([-np.logspace(-12, -3, 40), [0.0], np.logspace(-12, -3, 40)])
    pts = []
    for r in (1.0, 17.3, 80.0):
        for d in offs:
            a = np.radians(h + d)
            pts.append([r * np.cos(a), r * np.sin(a), 0.0, 0.5])
            pts.append([r * np.cos(a), -r * np.sin(a), 0.1, 0.5])
            e = np.radians(v + d)
            pts.append([r * np.cos(e), 0.0, r * np.sin(e), 0.5])
            pts.append([r * np.cos(e), 0.0, -r * np.sin(e), 0.5])
    env = np.array(pts)
    pose = {"position": np.zeros(3), "orientation": np.zeros(3)}
    ref = R.scan_environment(env, pose, sim.config)
    out = sim.scan_environment(env, pose)
    assert out.shape == ref.shape
    assert_scaled_close(out, ref, scale_of(ref[:, :3]), what="fov edges")


def test_scan_then_align_round_trip_recovers_the_scene(mc, gpu_ctx):
    """SURVEY §4 property: scan applies R^T (p - t) (LMC:726-728) and alignment R p + t, so without
    noise every aligned point of every frame is a scene point.
    1200 frames of the urban run over a 60k-point scene, all points checked (float64 rows: within a
    few ulp of the scene point)."""
    cfg = dict(CFGS["urban_complex"], lidar_range_noise=0.0)
    sim = mc.LiDARMotionSimulator(cfg, context=gpu_ctx)
    tr = traj_of("urban_complex")
    env = synth_scene(21, 60_000)[:, :4]
    env[:, :2] += tr["position_gps"][0, :2]
    res = sim.simulate_frames(env, tr)
    from scipy.spatial import cKDTree
    tree = cKDTree(env[:, :3])
    total = 0
    for f, al in enumerate(res["aligned_pointclouds"]):
        if len(al) == 0:
            continue
        d, j = tree.query(al[:, :3])
        scale = np.linalg.norm(env[j, :3], axis=1) + np.linalg.norm(res["raw_scans"][f]["sensor_pose"]["position"])
        assert np.all(d <= 1e-12 * scale), f
        assert np.array_equal(al[:, 3], env[j, 3]), f
        total += len(al)
    assert total > 100_000


def test_frame_rotation_is_orthonormal(mc, gpu_ctx):
    """SURVEY §4 property: the per-frame R is a rotation (orthonormal, det 1) for arbitrary angles."""
    rng = np.random.default_rng(2)
    sim = mc.LiDARMotionSimulator(context=gpu_ctx)
    basis = np.array([[1.0, 0, 0, 0], [0, 1.0, 0, 0], [0, 0, 1.0, 0], [0, 0, 0, 0]])
    for _ in range(20):
        pose = {"translation": rng.normal(0, 100, 3), "rotation": rng.uniform(-4, 4, 3)}
        out = sim.transform_pointcloud(basis, pose)
        Rm = (out[:3, :3] - out[3, :3]).T
        np.testing.assert_allclose(Rm @ Rm.T, np.eye(3), atol=1e-12)
        assert abs(np.linalg.det(Rm) - 1.0) < 1e-12


def test_scan_noise_consumes_global_rng_like_reference(mc, gpu_ctx):
    cfg = dict(points_per_frame=3000, lidar_range_noise=0.02)
    sim = mc.LiDARMotionSimulator(cfg, context=gpu_ctx)
    env = synth_scene(3, 100_000)
    poses = [{"position": np.array([0.0, 0, 1]), "orientation": np.array([0, 0, a])} for a in (0.0, 1.0, 2.5)]
    np.random.seed(123)
    ref = [R.scan_environment(env, p, sim.config) for p in poses]
    after_ref = np.random.random()
    np.random.seed(123)
    out = [sim.scan_environment(env, p) for p in poses]
    assert np.random.random() == after_ref
    for o, r in zip(out, ref):
        assert_scaled_close(o, r, scale_of(r[:, :3]), what="noisy")


def test_scene_cache_two_simulators_one_context_and_in_place_edits(mc, gpu_ctx):
    """The scene lives on the context: two simulators sharing it, alternating two scenes, and
    in-place edits of one scene array (a row permutation, a sum-preserving +d / -d move) must each
    scan the scene passed in (LMC:701-770), never a stale upload."""
    cfg = dict(points_per_frame=4000, lidar_range_noise=0.0)
    a = mc.LiDARMotionSimulator(cfg, context=gpu_ctx)
    b = mc.LiDARMotionSimulator(cfg, context=gpu_ctx)
    env1 = synth_scene(31, 50_000)
    env2 = synth_scene(32, 50_000)
    pose = {"position": np.array([1.0, -2.0, 0.5]), "orientation": np.array([0.01, -0.02, 0.7])}

    def check(sim, env, what):
        ref = R.scan_environment(env, pose, sim.config)
        out = sim.scan_environment(env, pose)
        assert out.shape == ref.shape, what
        assert_scaled_close(out, ref, scale_of(ref[:, :3]) + 1e-3, what=what)
        assert np.array_equal(out[:, 3], ref[:, 3]), what

    for rep in range(2):
        check(a, env1, f"A scene 1 rep {rep}")
        check(b, env2, f"B scene 2 rep {rep}")
    # same array object, rows permuted in place: changes the subsample and the output order
    perm = np.random.default_rng(4).permutation(len(env1))
    env1[:] = env1[perm]
    check(a, env1, "A scene 1 permuted in place")
    # sum-preserving edit of two visible points
    vis = R.scan_environment(env1, pose, dict(a.config, points_per_frame=10 ** 9))
    assert len(vis) > 2
    j = np.flatnonzero(np.isin(env1[:, 3], vis[:2, 3]))[:2]
    env1[j[0], 0] += 0.25
    env1[j[1], 0] -= 0.25
    check(a, env1, "A scene 1 +d/-d")
    check(b, env2, "B scene 2 after A's edits")


def test_scan_emit_refuses_stale_scene(mc, gpu_ctx):
    """mc_scan_emit_f64 after mc_set_environment without a new mc_scan_count: MC_ERR_STATE."""
    sim = mc.LiDARMotionSimulator(dict(points_per_frame=100, lidar_range_noise=0.0), context=gpu_ctx)
    env = synth_scene(7, 5000)
    gpu_ctx.set_environment(env)
    gpu_ctx.set_trajectory([0.0], np.zeros((1, 3)), np.zeros((1, 3)))
    counts, _ = gpu_ctx._scan_count([0.0], sim.config, "direct", np.random)
    assert counts.sum() > 0
    gpu_ctx.set_environment(env[::-1])
    buf = gpu_ctx.device_buffer(int(counts.sum()) * 32)
    try:
        rc = gpu_ctx.lib.mc_scan_emit_f64(gpu_ctx.handle, None, buf.ptr, None)
        assert rc == mc._lib.MC_ERR_STATE
    finally:
        buf.close()


def test_scan_one_point_in_range_bitwise(mc, gpu_ctx):
    """LMC:728 with exactly one scene point inside range_max: numpy's (R.T @ d.T).T is a (3,3) @ (3,1)
    product (R.T F-contiguous), which keeps the multi-row ascending FMA chain (tools/fma_order.py), so
    the device's sensor-frame point equals the reference expression bit for bit."""
    from scipy.spatial.transform import Rotation
    sim = mc.LiDARMotionSimulator({"lidar_range_noise": 0.0}, context=gpu_ctx)
    rng = np.random.default_rng(17)
    hits = 0
    for _ in range(200):
        pos = rng.uniform(-50, 50, 3)
        rpy = rng.uniform(-np.pi, np.pi, 3)
        Rm = Rotation.from_euler("xyz", rpy).as_matrix()
        r = rng.uniform(2, 80)        # a sensor-frame point well inside the FOV, carried to the world
        loc = np.array([r, r * rng.uniform(-0.3, 0.3), r * rng.uniform(-0.3, 0.3)])
        env = np.array([[*(pos + Rm @ loc), 0.37], [*(pos + 500.0), 0.5], [*(pos - 700.0), 0.6]])
        out = sim.scan_environment(env, {"position": pos, "orientation": rpy})
        envf = env[:1]
        want = (Rm.T @ (envf[:, :3] - pos).T).T          # the reference's expression, one row
        assert out.shape == (1, 4)
        assert np.array_equal(out[:, :3], want), (out[:, :3] - want)
        hits += 1
    assert hits == 200
