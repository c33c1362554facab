"""GPU parity: the HIP path through the C-ABI vs the oracle and the reference's golden vectors.

Tolerance (north_star: <= 1e-5 relative per coordinate), conftest.assert_scaled_close: strict per
coordinate |gpu - ref| <= 1e-5 * |ref| (floor at 1e-9 * (|p| + |t|)) wherever the input is made of
float32 values — the float32 columns then hold the reference's exact inputs, and the kernels' float64
arithmetic leaves only the final rounding (2^-24).  Random inputs are drawn as float32 values
(``f32``) for that reason.  Reference float64 data staged into float32 columns (golden frames of the
reference run) is compared at the scaled bar |gpu - ref| <= 1e-5 * (|p| + |t|) and,
strictly, against the oracle on the same float32-rounded inputs.
"""
import os

import numpy as np
import pytest

from conftest import assert_scaled_close, golden, scale_of
from oracle import restatement as R
from oracle import synth

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


def f32(a):
    """float64 array of float32 values (what a float32 batch column holds exactly)."""
    return np.asarray(a, dtype=np.float64).astype(np.float32).astype(np.float64)


def traj_of(name):
    g = golden(f"lmc_traj_{name}.npz")
    return {k: g[k] for k in g.files}


# ---------------------------------------------------------------------------------------------
# Path A
# ---------------------------------------------------------------------------------------------
def test_transform_pointcloud_known_answers(mc, gpu_ctx):
    g = golden("lmc_kat.npz")
    sim = mc.LiDARMotionSimulator(context=gpu_ctx)
    pts = g["points"]
    for i in range(int(g["n_cases"])):
        before = pts.copy()
        out = sim.transform_pointcloud(pts, {"translation": g[f"t{i}"], "rotation": g[f"r{i}"]})
        assert out.dtype == np.float64 and out.shape == (len(pts), 4)
        assert np.array_equal(pts, before)   # input untouched
        assert_scaled_close(out[:, :3], g[f"out{i}"][:, :3], scale_of(pts[:, :3], g[f"t{i}"]), what=f"kat{i}")
        # bit for bit: scipy's R (rot.cpp) and numpy's matmul accumulation order (frame_apply)
        assert np.array_equal(out, g[f"out{i}"]), (i, int(np.count_nonzero(out != g[f"out{i}"])))
    # one frame above the zero-copy size: the DMA row pipeline, bitwise too (the reference's output
    # recorded by sha256 and every 1000th row; the points regenerated from their seed)
    import hashlib
    brng = np.random.default_rng(2024)
    big = np.column_stack([brng.uniform(-90, 90, (40_000, 3)), brng.uniform(0, 1, 40_000)])
    bo = sim.transform_pointcloud(big, {"translation": g["t3"], "rotation": g["r3"]})
    assert np.array_equal(bo[::1000], g["big/rows"])
    assert hashlib.sha256(np.ascontiguousarray(bo).tobytes()).digest() == g["big/sha256"].tobytes()
    assert sim.transform_pointcloud(np.zeros((0, 4)), {"translation": np.zeros(3), "rotation": np.zeros(3)}).shape == (0, 4)
    # one-point frames: numpy's matrix-vector product (another summation order) reproduced as well,
    # alone and inside a batch of one-point frames
    for i in range(int(g["n_cases"])):
        tf = {"translation": g[f"t{i}"], "rotation": g[f"r{i}"]}
        one = g[f"one{i}"]
        assert np.array_equal(sim.transform_pointcloud(pts[5:6], tf), one[5:6]), i
        got = np.vstack(sim.align_frames([pts[j:j + 1] for j in range(len(pts))], [tf] * len(pts)))
        assert np.array_equal(got, one), (i, int(np.count_nonzero(got != one)))
    with pytest.raises(IndexError):
        sim.transform_pointcloud(np.zeros((5, 3)), {"translation": np.zeros(3), "rotation": np.zeros(3)})
    with pytest.raises(IndexError):
        sim.transform_pointcloud(np.zeros(4), {"translation": np.zeros(3), "rotation": np.zeros(3)})


@pytest.mark.parametrize("name", list(SCEN))
def test_run_alignment_matches_reference_frames(mc, gpu_ctx, name):
    g = golden("lmc_frames.npz")
    tr = traj_of(name)
    sim = mc.LiDARMotionSimulator(dict(CFGS[name]), context=gpu_ctx)
    times = sim.lidar_times()
    fids = SCEN[name]
    scans = [g[f"{name}/{f}/points_local"] for f in fids]
    out = sim.run_alignment(scans, tr, times[fids])
    for f, o in zip(fids, out):
        ref = g[f"{name}/{f}/aligned"]
        assert o.shape == ref.shape
        assert_scaled_close(o[:, :3], ref[:, :3], scale_of(g[f"{name}/{f}/points_local"][:, :3],
                                                           g[f"{name}/{f}/position"]), what=f"{name}/{f}")
        assert np.array_equal(o, ref), (name, f, int(np.count_nonzero(o != ref)))   # the reference's bits
    merged = sim.merge_aligned(out)
    assert merged.shape == (sum(len(s) for s in scans), 4)


def test_run_alignment_large_results_through_recycled_blocks(mc, gpu_ctx):
    """run_alignment over > 1 M rows (the two-stream row pipeline) into runtime.HostPool blocks: the
    first result in a fresh block, the next ones in the recycled block once the previous result is
    dropped.  Every call bitwise equal to the reference's op sequence (scipy R, numpy matmul),
    ragged frames and a wider (5-column) frame included."""
    from oracle import restatement as R
    rng = np.random.default_rng(12)
    counts = [300_000, 1, 0, 777_777, 250_001]
    scans = [np.column_stack([rng.normal(0, 40, (n, 3)), rng.uniform(0, 1, n)]) for n in counts]
    scans[3] = np.column_stack([scans[3], np.full(len(scans[3]), 7.0)])      # a 5-column frame
    sim = mc.LiDARMotionSimulator(dict(CFGS["urban_complex"]), context=gpu_ctx)
    tr = traj_of("urban_complex")
    times = sim.lidar_times()[[3, 4, 5, 6, 7]]
    idx = R.select_pose_index(tr["time"], times)
    want = [R.transform_pointcloud_ref_ops(s, {"translation": tr["position_gps"][k],
                                               "rotation": tr["orientation_imu"][k]}) for s, k in zip(scans, idx)]
    pool = mc.runtime.host_pool()
    for call in range(3):
        out = sim.run_alignment(scans, tr, times)
        for f, (o, w) in enumerate(zip(out, want)):
            assert np.array_equal(o, w), (call, f, int(np.count_nonzero(o != w)))
        del out, o
        assert pool.idle_bytes() >= sum(counts) * 32          # the block is back for the next call


def test_align_frames_ragged_batch(mc, gpu_ctx):
    rng = np.random.default_rng(1)
    counts = [0, 1, 2, 3, 4, 5, 7, 4096, 0, 2049, 2047, 1023, 100_003]
    frames = [np.column_stack([rng.uniform(-90, 90, (n, 3)), rng.uniform(0, 1, n)]) for n in counts]
    tfs = [{"translation": rng.normal(0, 500, 3), "rotation": rng.uniform(-np.pi, np.pi, 3)} for _ in counts]
    sim = mc.LiDARMotionSimulator(context=gpu_ctx)
    out = sim.align_frames(frames, tfs)
    for f, t, o in zip(frames, tfs, out):
        ref = R.transform_pointcloud(f, t)
        assert o.shape == ref.shape
        assert_scaled_close(o[:, :3], ref[:, :3], scale_of(f[:, :3], t["translation"]))


def test_frame_mode_grid_stride_and_inplace(mc, gpu_ctx):
    counts = np.array([30_000, 77_777, 1, 50_000])
    tr = traj_of("urban_complex")
    b = gpu_ctx.batch(counts, with_time=False)
    b.synth(seed=3, frame_id_base=0)
    b.set_frame_times([0.0, 0.35, 7.3, 119.99])
    gpu_ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    out1 = gpu_ctx.deskew(b, mode="frame").download_aos()
    gpu_ctx.set_max_grid(37)
    try:
        out2 = gpu_ctx.deskew(b, mode="frame").download_aos()
    finally:
        gpu_ctx.set_max_grid(0)
    assert np.array_equal(out1, out2)
    gpu_ctx.deskew(b, b, mode="frame")   # in place
    assert np.array_equal(b.download_aos(), out1)


# ---------------------------------------------------------------------------------------------
# synthetic generator + full-size properties
# ---------------------------------------------------------------------------------------------
def test_device_generator_bit_identical(mc, gpu_ctx):
    counts = np.array([100_000, 3, 0, 20_001])
    b = gpu_ctx.batch(counts, with_time=True)
    b.synth(seed=0, frame_id_base=1000)
    x, y, z, i = b.download_columns()
    t = b.download_time()
    hx, hy, hz, hi, ht = synth.synth_batch(counts, seed=0, frame_id_base=1000)
    for a, h in zip((x, y, z, i, t), (hx, hy, hz, hi, ht)):
        assert np.array_equal(a, h)
    g = golden("synth.npz")
    assert np.array_equal(x[:4096], g["x"]) and np.array_equal(t[:4096], g["t"])
    np.testing.assert_allclose(b.checksum(), [c.astype(np.float64).sum() for c in (hx, hy, hz, hi, ht)], rtol=1e-12)


def _c2_batch(mc, ctx, frames=600, n=100_000, with_time=True):
    sim = mc.LiDARMotionSimulator(dict(CFGS["urban_complex"]), context=ctx)
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:frames]
    b = ctx.batch(np.full(frames, n), with_time=with_time)
    b.synth(seed=0, frame_id_base=1000)
    b.set_frame_times(times)
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    return b, tr, times


def test_full_size_c2_frame_mode_all_points(mc, gpu_ctx):
    """BASELINE config 2 (600 x 100k) in frame mode, every point checked against the oracle."""
    b, tr, times = _c2_batch(mc, gpu_ctx, with_time=False)
    out = gpu_ctx.deskew(b, mode="frame")
    ox, oy, oz, oi = out.download_columns()
    hx, hy, hz, hi, _ = synth.synth_batch(b.counts, seed=0, frame_id_base=1000)
    idx = R.select_pose_index(tr["time"], times)
    Rm = R.euler_xyz_matrix(tr["orientation_imu"][idx])
    T = tr["position_gps"][idx]
    n = 100_000
    worst = 0.0
    for f in range(0, 600, 1):
        s = slice(f * n, (f + 1) * n)
        p = np.stack([hx[s], hy[s], hz[s]], axis=1).astype(np.float64)
        ref = p @ Rm[f].T + T[f]
        got = np.stack([ox[s], oy[s], oz[s]], axis=1)
        worst = max(worst, assert_scaled_close(got, ref, scale_of(p, T[f]), what=f"frame {f}"))
    assert np.array_equal(oi, hi)


@pytest.mark.parametrize("mode", ["pose_slerp", "imu"])
def test_full_size_c2_per_point_modes_all_points(mc, gpu_ctx, mode):
    """BASELINE config 2 (600 x 100k) in the per-point modes, every point checked against the
    oracle (frames in chunks on a thread pool: numpy releases the GIL), plus the rotation-norm
    invariant of Path B over all 60M points."""
    from concurrent.futures import ThreadPoolExecutor

    b, tr, times = _c2_batch(mc, gpu_ctx)
    ts = gyro = starts = None
    if mode == "imu":
        ts, gyro = mc.trajectory.imu_from_trajectory(tr, 200.0)
        gpu_ctx.set_imu(ts, gyro)
        starts = (times * 1e9).astype(np.int64)
        b.set_frame_starts(starts)
    out = gpu_ctx.deskew(b, mode=mode)
    ox, oy, oz, oi = out.download_columns()
    hx, hy, hz, hi, ht = synth.synth_batch(b.counts, seed=0, frame_id_base=1000)
    assert np.array_equal(oi, hi)
    n, F, per = 100_000, 600, 10

    def chunk(f0):
        s = slice(f0 * n, (f0 + per) * n)
        p = np.stack([hx[s], hy[s], hz[s]], axis=1).astype(np.float64)
        got = np.stack([ox[s], oy[s], oz[s]], axis=1)
        fr = np.repeat(np.arange(f0, f0 + per), n)
        t = ht[s].astype(np.int64)
        if mode == "pose_slerp":
            Rm, pos = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"], times[fr] + t * 1e-9)
            ref = np.einsum("nij,nj->ni", Rm, p) + pos
            sc = scale_of(p, pos)
        else:   # R.compensate_arrays with a per-point frame start
            w = R.imu_interpolate_gyro(ts, gyro, starts[fr] + t)
            Rm = R.euler_xyz_matrix(w * (t * 1e-9)[:, None])
            ref = np.einsum("nji,nj->ni", Rm, p)
            sc = scale_of(p)
        return assert_scaled_close(got, ref, sc, what=f"{mode} frames {f0}..{f0 + per - 1}")

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as pool:
        worst = max(pool.map(chunk, range(0, F, per)))
    assert worst <= 1e-5
    if mode == "imu":   # rotation only: norms preserved over the full 60M points
        nin = np.sqrt(hx.astype(np.float64) ** 2 + hy.astype(np.float64) ** 2 + hz.astype(np.float64) ** 2)
        nout = np.sqrt(ox.astype(np.float64) ** 2 + oy.astype(np.float64) ** 2 + oz.astype(np.float64) ** 2)
        assert np.max(np.abs(nout - nin) / nin) < 1e-5


def test_config5_shape_1m_point_frames_all_points(mc, gpu_ctx):
    """BASELINE config 5's per-GPU shape (dense 1M-point frames; 150 of them = 1200 frames / 8 GPUs)
    in the headline SLERP mode: every one of the 150M points against the oracle."""
    from concurrent.futures import ThreadPoolExecutor

    F, n = 150, 1_000_000
    b, tr, times = _c2_batch(mc, gpu_ctx, frames=F, n=n)
    out = gpu_ctx.deskew(b, mode="pose_slerp")
    ox, oy, oz, oi = out.download_columns()
    out.close()
    b.close()
    hx, hy, hz, hi, ht = synth.synth_batch(np.full(F, n), seed=0, frame_id_base=1000)
    assert np.array_equal(oi, hi)

    def check(f):
        s = slice(f * n, (f + 1) * n)
        p = np.stack([hx[s], hy[s], hz[s]], axis=1).astype(np.float64)
        Rm, pos = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"], times[f] + ht[s] * 1e-9)
        ref = np.einsum("nij,nj->ni", Rm, p) + pos
        return assert_scaled_close(np.stack([ox[s], oy[s], oz[s]], axis=1), ref, scale_of(p, pos), what=f"frame {f}")

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as pool:
        assert max(pool.map(check, range(F))) <= 1e-5


def test_max_size_c4_on_one_gpu_past_int32_indices(mc, gpu_ctx):
    """BASELINE config 4's whole job (6000 x 100k, urban poses over 600 s) on ONE device: 600 M
    points, 3.0 G values in the 5-column input (past 2^31), 12 GB in + 9.6 GB out.  SLERP into a
    4-column batch, then frame mode in place on that output; frames at both ends and across the
    2^31-value boundary are checked against the oracle."""
    F, n = 6000, 100_000
    cfg = dict(CFGS["urban_complex"], duration=600.0)
    sim = mc.LiDARMotionSimulator(cfg, context=gpu_ctx)
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:F]
    assert len(times) == F
    b = gpu_ctx.batch(np.full(F, n), with_time=True)
    b.synth(seed=7, frame_id_base=1000)
    b.set_frame_times(times)
    gpu_ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    out = gpu_ctx.deskew(b, gpu_ctx.batch(b.counts), mode="pose_slerp")
    b.close()
    g = np.stack(out.download_columns()[:3], axis=1)
    out.set_frame_times(times)
    gpu_ctx.deskew(out, out, mode="frame")
    h = np.stack(out.download_columns()[:3], axis=1)
    idx = R.select_pose_index(tr["time"], times)
    edge = (2 ** 31) // (5 * n)          # first frames whose t_ns column lies past 2^31 values
    for f in [0, 1, edge - 1, edge, edge + 1, 4297, F - 2, F - 1]:
        x, y, z, _, t = synth.synth_frame(n, 7, 1000 + f)
        p = np.stack([x, y, z], axis=1).astype(np.float64)
        s = slice(f * n, (f + 1) * n)
        ref = R.deskew_pose_slerp(p, t, times[f], tr)
        _, pos = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"], times[f] + t * 1e-9)
        assert_scaled_close(g[s], ref, scale_of(p, pos), what=f"slerp frame {f}")
        k = idx[f]
        gp = g[s].astype(np.float64)
        ref2 = R.transform_pointcloud(np.column_stack([gp, np.zeros(n)]),
                                      {"translation": tr["position_gps"][k], "rotation": tr["orientation_imu"][k]})
        assert_scaled_close(h[s], ref2[:, :3], scale_of(gp, tr["position_gps"][k]), what=f"frame {f}")
    out.close()


def _scenario_batch(mc, ctx, name, frames, n, seed):
    sim = mc.LiDARMotionSimulator(dict(CFGS[name]), context=ctx)   # seeds np.random (LMC:288): noise on
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:frames]
    b = ctx.batch(np.full(frames, n), with_time=True)
    b.synth(seed=seed, frame_id_base=1000)
    b.set_frame_times(times)
    b.set_frame_starts((times * 1e9).astype(np.int64))
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    ts, gyro = mc.trajectory.imu_from_trajectory(tr, 200.0)
    ctx.set_imu(ts, gyro)
    return b, tr, times, ts, gyro


def _check_frames(mc, ctx, b, tr, times, ts, gyro, mode, frames_to_check, n, seed):
    out = ctx.deskew(b, mode=mode)
    ox, oy, oz, oi = out.download_columns()
    hx, hy, hz, hi, ht = synth.synth_batch(b.counts, seed=seed, frame_id_base=1000)
    assert np.array_equal(oi, hi)
    idx = R.select_pose_index(tr["time"], times)

    def check(f):
        s = slice(f * n, (f + 1) * n)
        p = np.stack([hx[s], hy[s], hz[s]], axis=1).astype(np.float64)
        got = np.stack([ox[s], oy[s], oz[s]], axis=1)
        if mode == "frame":
            k = idx[f]
            ref = R.transform_pointcloud(np.column_stack([p, hi[s]]),
                                         {"translation": tr["position_gps"][k], "rotation": tr["orientation_imu"][k]})[:, :3]
            sc = scale_of(p, tr["position_gps"][k])
        elif mode == "pose_slerp":
            ref = R.deskew_pose_slerp(p, ht[s], times[f], tr)
            _, pos = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"], times[f] + ht[s] * 1e-9)
            sc = scale_of(p, pos)
        else:
            st = int(times[f] * 1e9)
            ref = R.compensate_arrays(p, st + ht[s].astype(np.int64), st, ts, gyro)
            sc = scale_of(p)
        return assert_scaled_close(got, ref, sc, what=f"{mode} frame {f}")

    from concurrent.futures import ThreadPoolExecutor   # numpy releases the GIL
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as pool:
        return max(pool.map(check, frames_to_check))


@pytest.mark.parametrize("mode", ["frame", "pose_slerp", "imu"])
def test_config1_highway_10x20k_all_points(mc, gpu_ctx, mode):
    """BASELINE config 1 (highway_simple, linear, 10 frames x 20k points): every point, every mode."""
    b, tr, times, ts, gyro = _scenario_batch(mc, gpu_ctx, "highway_simple", 10, 20_000, seed=5)
    _check_frames(mc, gpu_ctx, b, tr, times, ts, gyro, mode, range(10), 20_000, seed=5)


@pytest.mark.parametrize("mode", ["pose_slerp", "frame", "imu"])
def test_config3_parking_600x100k_all_points(mc, gpu_ctx, mode):
    """BASELINE config 3 (parking_detailed, circular, IMU/GPS noise on, SLERP-heavy): 600 x 100k,
    every point of every frame (the run crosses the yaw wrap) in every mode."""
    b, tr, times, ts, gyro = _scenario_batch(mc, gpu_ctx, "parking_detailed", 600, 100_000, seed=9)
    _check_frames(mc, gpu_ctx, b, tr, times, ts, gyro, mode, range(600), 100_000, seed=9)


# ---------------------------------------------------------------------------------------------
# per-point SLERP mode
# ---------------------------------------------------------------------------------------------
def _batch_deskew(ctx, frames, t_ns, mode, times=None, starts=None, tr=None):
    """The device-batch path (float32 columns, k_deskew_points) over host frames: what the bench
    runs; the drop-in methods take the float64 rows path (k_points_f64) instead.  SLERP: ``tr`` is
    uploaded here (the context keeps whatever table the last call set)."""
    if tr is not None:
        ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    b = ctx.batch(np.array([len(f) for f in frames]), with_time=True)
    b.upload_aos(np.concatenate([np.column_stack([f[:, :3], f[:, 3] if f.shape[1] > 3 else np.zeros(len(f))])
                                 for f in frames]))
    b.upload_time(np.concatenate([np.asarray(t, np.int64) for t in t_ns]))
    if times is not None:
        b.set_frame_times(times)
    if starts is not None:
        b.set_frame_starts(starts)
    return b.split(ctx.deskew(b, mode=mode).download_aos())


def test_slerp_matches_scipy_golden_across_yaw_wrap(mc, gpu_ctx):
    g = golden("slerp.npz")
    tr = {"time": g["time"], "position_gps": g["position_gps"], "orientation_imu": g["orientation_imu"]}
    t_frame = float(g["tq"][0])
    t_ns = np.round((g["tq"] - t_frame) * 1e9).astype(np.int64)
    sim = mc.LiDARMotionSimulator(context=gpu_ctx)
    pts = np.column_stack([g["xyz"], np.linspace(0, 1, len(g["xyz"]))])
    out = sim.deskew_frames([pts], [t_ns], tr, times=[t_frame])[0]
    tq = t_frame + t_ns * 1e-9
    _, pos = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"], tq)
    # the drop-in computes in float64 on the float64 points: strict against the oracle and the golden
    ref = R.deskew_pose_slerp(g["xyz"], t_ns, t_frame, tr)
    assert_scaled_close(out[:, :3], ref, scale_of(g["xyz"], pos), what="slerp vs oracle")
    assert_scaled_close(out[:, :3], g["out"], scale_of(g["xyz"], pos), what="slerp vs scipy golden")
    assert np.array_equal(out[:, 3], pts[:, 3])
    # the device-batch kernel holds float32 columns: strict against the oracle on those inputs
    bo = _batch_deskew(gpu_ctx, [pts], [t_ns], "pose_slerp", times=[t_frame], tr=tr)[0]
    assert_scaled_close(bo[:, :3], R.deskew_pose_slerp(f32(g["xyz"]), t_ns, t_frame, tr), scale_of(g["xyz"], pos),
                        what="batch slerp vs oracle")


def test_slerp_edge_cases_and_slow_path(mc, gpu_ctx):
    """Unsorted times, negative offsets, times beyond both ends of the pose table (clamp), a
    dense pose table so that one 1024-point sub-tile spans > 64 segments (out-of-line path)."""
    rng = np.random.default_rng(9)
    T = 4000
    time = np.linspace(0, 40, T)                      # 100 Hz pose table
    rpy = np.cumsum(rng.normal(0, 0.05, (T, 3)), axis=0)
    pos = np.cumsum(rng.normal(0, 0.2, (T, 3)), axis=0)
    tr = {"time": time, "position_gps": pos, "orientation_imu": rpy}
    counts = [5000, 3, 1024, 2500]
    frames = [f32(np.column_stack([rng.uniform(-90, 90, (n, 3)), rng.uniform(0, 1, n)])) for n in counts]
    t_ns = [rng.integers(-2_000_000_000, 2_000_000_000, counts[0]),          # spans 4 s: slow path
            np.array([-10**9, 0, 10**9]),
            np.sort(rng.integers(0, 100_000_000, 1024)),
            rng.integers(0, 100_000_000, 2500)]                                # unsorted
    times = np.array([1.0, 0.2, 20.0, 39.95])                                 # frame 3 runs off the end
    sim = mc.LiDARMotionSimulator(context=gpu_ctx)
    for path, out in (("float64 rows", sim.deskew_frames(frames, t_ns, tr, times)),
                      ("batch", _batch_deskew(gpu_ctx, frames, t_ns, "pose_slerp", times=times, tr=tr))):
        for f in range(len(counts)):
            ref = R.deskew_pose_slerp(frames[f][:, :3], t_ns[f], times[f], tr)
            _, p = R.slerp_pose(time, pos, rpy, times[f] + np.asarray(t_ns[f]) * 1e-9)
            assert_scaled_close(out[f][:, :3], ref, scale_of(frames[f][:, :3], p), what=f"{path} frame {f}")


@pytest.mark.parametrize("mode", ["pose_slerp", "imu"])
def test_wide_frames_take_subtile_windows(mc, gpu_ctx, mode):
    """Frames spanning many pose / IMU segments (100 Hz poses, 1 kHz IMU): time-ordered frames use
    per-sub-tile windows of 1-2 segments (SGPR path, incl. sub-tiles straddling a boundary), a
    shuffled frame the sub-tile LDS window, a 3-s frame the out-of-line search; all vs the oracle."""
    rng = np.random.default_rng(12)
    T = 4000
    time = np.linspace(0, 40, T)
    tr = {"time": time, "position_gps": np.cumsum(rng.normal(0, 0.2, (T, 3)), axis=0),
          "orientation_imu": np.cumsum(rng.normal(0, 0.05, (T, 3)), axis=0)}
    counts = [50_000, 50_000, 20_000, 4096, 7]
    t_ns = [np.sort(rng.integers(0, 100_000_000, counts[0])),
            np.arange(counts[1]) * 2000,                                     # exact 2 us spacing
            rng.permutation(np.arange(counts[2]) * 5000),                     # shuffled
            rng.integers(-1_500_000_000, 1_500_000_000, counts[3]),           # 3 s span
            np.array([0, 1, 2, 99_999_999, 50_000_000, 3, 4])]
    frames = [f32(np.column_stack([rng.uniform(-90, 90, (n, 3)), rng.uniform(0, 1, n)])) for n in counts]
    times = np.array([2.0, 10.005, 20.0, 30.0, 35.0])
    sim = mc.LiDARMotionSimulator(context=gpu_ctx)
    if mode == "pose_slerp":
        out = _batch_deskew(gpu_ctx, frames, t_ns, "pose_slerp", times=times, tr=tr)
        o64 = sim.deskew_frames(frames, t_ns, tr, times)
        for f in range(len(counts)):
            ref = R.deskew_pose_slerp(frames[f][:, :3], t_ns[f], times[f], tr)
            _, p = R.slerp_pose(time, tr["position_gps"], tr["orientation_imu"], times[f] + np.asarray(t_ns[f]) * 1e-9)
            assert_scaled_close(out[f][:, :3], ref, scale_of(frames[f][:, :3], p), what=f"frame {f}")
            assert_scaled_close(o64[f][:, :3], ref, scale_of(frames[f][:, :3], p), what=f"float64 rows frame {f}")
    else:
        ts = np.arange(0, 40_000_000_000, 1_000_000, dtype=np.int64)            # 1 kHz
        gyro = rng.normal(0, 0.5, (len(ts), 3))
        starts = (times * 1e9).astype(np.int64)
        b = gpu_ctx.batch(np.array(counts), with_time=True)
        b.upload_aos(np.concatenate(frames))
        b.upload_time(np.concatenate(t_ns).astype(np.int32))
        b.set_frame_starts(starts)
        gpu_ctx.set_imu(ts, gyro)
        got = b.split(gpu_ctx.deskew(b, mode="imu").download_aos())
        for f in range(len(counts)):
            ref = R.compensate_arrays(frames[f][:, :3], starts[f] + np.asarray(t_ns[f], np.int64), starts[f], ts, gyro)
            assert_scaled_close(got[f][:, :3], ref, scale_of(frames[f][:, :3]), what=f"imu frame {f}")


@pytest.mark.parametrize("mode", ["pose_slerp", "imu"])
def test_per_point_modes_pass_t_ns_through(mc, gpu_ctx, mode):
    """CSIM:1472 keeps each point's timestamp: out-of-place deskew into a batch with t_ns copies
    the column from inside the kernel (fast and out-of-line paths); in place leaves it as is; the
    result equals the in-place run and a 4-column output batch."""
    rng = np.random.default_rng(4)
    T = 4000
    time = np.linspace(0, 40, T)
    tr = {"time": time, "position_gps": np.cumsum(rng.normal(0, 0.2, (T, 3)), axis=0),
          "orientation_imu": np.cumsum(rng.normal(0, 0.05, (T, 3)), axis=0)}
    counts = np.array([5000, 3, 0, 1024, 70_001])
    t_ns = np.concatenate([rng.integers(-2_000_000_000, 2_000_000_000, counts[0]),   # slow path
                           rng.integers(0, 100_000_000, int(counts[1:].sum()))]).astype(np.int32)
    pts = np.column_stack([rng.uniform(-90, 90, (int(counts.sum()), 3)), rng.uniform(0, 1, int(counts.sum()))])
    b = gpu_ctx.batch(counts, with_time=True)
    b.upload_aos(pts)
    b.upload_time(t_ns)
    if mode == "pose_slerp":
        gpu_ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
        b.set_frame_times(np.array([1.0, 0.2, 5.0, 20.0, 39.0]))
    else:
        ts = np.arange(0, 40_000_000_000, 5_000_000, dtype=np.int64)
        gpu_ctx.set_imu(ts, rng.normal(0, 0.3, (len(ts), 3)))
        b.set_frame_starts(np.array([3, 1, 5, 20, 30], np.int64) * 10**9)
    out_t = gpu_ctx.deskew(b, gpu_ctx.batch(counts, with_time=True), mode=mode)
    out_4 = gpu_ctx.deskew(b, gpu_ctx.batch(counts), mode=mode)
    got = out_t.download_aos()
    assert np.array_equal(out_t.download_time(), t_ns)
    assert np.array_equal(out_4.download_aos(), got)
    gpu_ctx.deskew(b, b, mode=mode)
    assert np.array_equal(b.download_aos(), got)
    assert np.array_equal(b.download_time(), t_ns)


def test_slerp_single_pose_table(mc, gpu_ctx):
    tr = {"time": np.array([3.0]), "position_gps": np.array([[1.0, 2.0, 3.0]]),
          "orientation_imu": np.array([[0.1, -0.2, 2.5]])}
    pts = f32(np.column_stack([np.random.default_rng(2).normal(0, 30, (100, 3)), np.zeros(100)]))
    sim = mc.LiDARMotionSimulator(context=gpu_ctx)
    out = sim.deskew_frames([pts], [np.arange(100) * 10**6], tr, times=[0.0])[0]
    ref = R.transform_pointcloud(pts, {"translation": tr["position_gps"][0], "rotation": tr["orientation_imu"][0]})
    assert_scaled_close(out[:, :3], ref[:, :3], scale_of(pts[:, :3], tr["position_gps"][0]))


# ---------------------------------------------------------------------------------------------
# Path B
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("case", ["mid", "before", "after", "dup", "spike", "noimu"])
def test_compensate_point_cloud_matches_reference(mc, gpu_ctx, case):
    g = golden("csim_pathb.npz")
    comp = mc.MotionCompensator({}, context=gpu_ctx)
    imu = [mc.IMUData(int(t), *map(float, gy), *map(float, ac))
           for t, gy, ac in zip(g[f"{case}/imu_ts"], g[f"{case}/imu_gyro"], g[f"{case}/imu_accel"])]
    xyz = g[f"{case}/xyz"]
    pts = [mc.LiDARPoint(float(p[0]), float(p[1]), float(p[2]), int(i), int(t), int(r), int(tg))
           for p, i, t, r, tg in zip(xyz, g[f"{case}/intensity"], g[f"{case}/ts"], g[f"{case}/ring"],
                                     g[f"{case}/tag"])]
    out = comp.compensate_point_cloud(pts, imu, int(g[f"{case}/frame_start"]), 100_000_000)
    if case == "noimu":
        assert out is pts
        return
    got = np.array([[p.x, p.y, p.z] for p in out])
    # float64 arithmetic on the reference's own float64 points: strict against its output and the oracle
    assert_scaled_close(got, g[f"{case}/out_xyz"], scale_of(xyz), what=case)
    ref = R.compensate_arrays(xyz, g[f"{case}/ts"], int(g[f"{case}/frame_start"]), g[f"{case}/imu_ts"],
                              g[f"{case}/imu_gyro"])
    assert_scaled_close(got, ref, scale_of(xyz), what=case + " vs oracle")
    meta = np.array([[p.intensity, p.timestamp, p.ring, p.tag] for p in out])
    assert np.array_equal(meta, g[f"{case}/out_meta"])


def test_compensator_disabled_and_driver(mc, gpu_ctx):
    g = golden("csim_pathb.npz")
    off = mc.MotionCompensator({"enable_motion_compensation": False}, context=gpu_ctx)
    pts = [mc.LiDARPoint(1.0, 2.0, 3.0, 5, 10, 0, 0)]
    assert off.compensate_point_cloud(pts, [mc.IMUData(0, 1, 1, 1, 0, 0, 0)], 0, 100_000_000) is pts
    comp = mc.MotionCompensator({}, context=gpu_ctx)
    imu = [mc.IMUData(int(t), *map(float, gy), 0.0, 0.0, 0.0) for t, gy in zip(g["mid/imu_ts"], g["mid/imu_gyro"])]
    frames = []
    for case in ("mid", "spike"):
        xyz = g[f"{case}/xyz"]
        frames.append({"timestamp": int(g[f"{case}/frame_start"]), "frame_duration_ns": 100_000_000,
                       "points": [mc.LiDARPoint(*map(float, p), int(i), int(t), 0, 0)
                                  for p, i, t in zip(xyz, g[f"{case}/intensity"], g[f"{case}/ts"])]})
    frames.append({"timestamp": 0, "frame_duration_ns": 100_000_000, "points": []})
    res = comp.apply_motion_compensation(frames, imu)
    assert all(r["motion_compensated"] for r in res) and res[2]["points"] == []
    for case, r in zip(("mid", "spike"), res):
        got = np.array([[p.x, p.y, p.z] for p in r["points"]])
        assert_scaled_close(got, g[f"{case}/out_xyz"], scale_of(g[f"{case}/xyz"]), what=case)


def test_apply_motion_compensation_reference_goldens_strict(mc, gpu_ctx):
    """CSIM:2086-2105 over every CSIM Path-B golden case at once: each case is a frame of one
    apply_motion_compensation call (one launch), checked strictly against the reference's own
    float64 output; metadata and record types pass through (CSIM:1467-1475)."""
    g = golden("csim_pathb.npz")
    cases = ["mid", "before", "after", "dup", "spike"]
    # every case shares the mid IMU list (the same table for all frames of a run)
    imu = [mc.IMUData(int(t), *map(float, gy), *map(float, ac))
           for t, gy, ac in zip(g["mid/imu_ts"], g["mid/imu_gyro"], g["mid/imu_accel"])]
    frames = []
    for case in cases:
        if not np.array_equal(g[f"{case}/imu_ts"], g["mid/imu_ts"]) or not np.array_equal(g[f"{case}/imu_gyro"], g["mid/imu_gyro"]):
            continue
        frames.append((case, {"timestamp": int(g[f"{case}/frame_start"]), "frame_duration_ns": 100_000_000,
                              "points": [mc.LiDARPoint(float(p[0]), float(p[1]), float(p[2]), int(i), int(t), int(r), int(tg))
                                         for p, i, t, r, tg in zip(g[f"{case}/xyz"], g[f"{case}/intensity"], g[f"{case}/ts"],
                                                                   g[f"{case}/ring"], g[f"{case}/tag"])]}))
    assert len(frames) >= 2
    comp = mc.MotionCompensator({}, context=gpu_ctx)
    res = comp.apply_motion_compensation([fr for _, fr in frames], imu)
    for (case, fr), r in zip(frames, res):
        got = np.array([[p.x, p.y, p.z] for p in r["points"]])
        assert_scaled_close(got, g[f"{case}/out_xyz"], scale_of(g[f"{case}/xyz"]), what=case)
        assert all(type(p) is mc.LiDARPoint for p in r["points"])
        meta = np.array([[p.intensity, p.timestamp, p.ring, p.tag] for p in r["points"]])
        assert np.array_equal(meta, g[f"{case}/out_meta"])


def test_points_f64_contract_and_edges(mc, gpu_ctx):
    """mc_deskew_points_f64: 3- and 5-column rows, empty frames in the middle, point times beyond
    int32 ns of their frame start (the batch path's limit), points before the first / after the last
    sample, the segment table rebuilt on a new IMU / trajectory upload, errors as the reference's."""
    rng = np.random.default_rng(21)
    ts = np.arange(0, 10_000_000_000, 5_000_000, dtype=np.int64)
    gyro = rng.normal(0, 0.8, (len(ts), 3))
    counts = np.array([700, 0, 3, 0, 40_000])                 # the last frame takes the staged (DMA) path
    starts = np.array([1, 2, 3, 4, 5], np.int64) * 1_000_000_000
    n = int(counts.sum())
    xyz = rng.uniform(-90, 90, (n, 3))
    t_rel = rng.integers(-3_000_000_000, 6_000_000_000, n)   # outside int32 ns and outside the IMU span
    gpu_ctx.set_imu(ts, gyro)
    for cols in (3, 5):
        pts = np.column_stack([xyz, rng.uniform(0, 1, (n, cols - 3))]) if cols > 3 else xyz
        out = mc.runtime.deskew_points_f64(gpu_ctx, "imu", counts, pts, t_rel, frame_start_ns=starts)
        offs = np.concatenate([[0], np.cumsum(counts)])
        for f in range(len(counts)):
            s = slice(offs[f], offs[f + 1])
            ref = R.compensate_arrays(xyz[s], starts[f] + t_rel[s], starts[f], ts, gyro)
            assert_scaled_close(out[s, :3], ref, scale_of(xyz[s]), what=f"cols {cols} frame {f}")
        assert np.array_equal(out[:, 3], pts[:, 3] if cols > 3 else np.zeros(n))
    gyro2 = gyro[::-1].copy()
    gpu_ctx.set_imu(ts, gyro2)                                # same length: the table must be rebuilt
    out = mc.runtime.deskew_points_f64(gpu_ctx, "imu", [n], xyz, t_rel, frame_start_ns=[starts[0]])
    assert_scaled_close(out[:, :3], R.compensate_arrays(xyz, starts[0] + t_rel, starts[0], ts, gyro2), scale_of(xyz))
    T = 300
    tr = {"time": np.linspace(0, 30, T), "position_gps": np.cumsum(rng.normal(0, 0.5, (T, 3)), axis=0),
          "orientation_imu": np.cumsum(rng.normal(0, 0.1, (T, 3)), axis=0)}
    gpu_ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    times = np.array([0.5, 1.0, 2.0, 3.0, 29.9])
    out = mc.runtime.deskew_points_f64(gpu_ctx, "pose_slerp", counts, xyz, t_rel, frame_times=times)
    offs = np.concatenate([[0], np.cumsum(counts)])
    for f in range(len(counts)):
        s = slice(offs[f], offs[f + 1])
        ref = R.deskew_pose_slerp(xyz[s], t_rel[s], times[f], tr)
        _, p = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"], times[f] + t_rel[s] * 1e-9)
        assert_scaled_close(out[s, :3], ref, scale_of(xyz[s], p), what=f"slerp frame {f}")
    with pytest.raises(IndexError):
        mc.runtime.deskew_points_f64(gpu_ctx, "imu", [n], xyz[:, :2], t_rel, frame_start_ns=[0])
    with pytest.raises(ValueError):
        mc.runtime.deskew_points_f64(gpu_ctx, "imu", [n + 1], xyz, t_rel, frame_start_ns=[0])
    with pytest.raises(ValueError):
        mc.runtime.deskew_points_f64(gpu_ctx, "frame", [n], xyz, t_rel, frame_start_ns=[0])
    assert mc.runtime.deskew_points_f64(gpu_ctx, "imu", [0, 0], np.zeros((0, 3)), [], frame_start_ns=[0, 0]).shape == (0, 4)


def test_compensator_sees_in_place_imu_edits(mc, gpu_ctx):
    """The reference reads the IMU list on every call (CSIM:1482-1516): editing interior samples of
    the same list object between calls (same length, same first / last timestamps) must change
    the result; a second compensator on the same context must not inherit a stale table."""
    g = golden("csim_pathb.npz")
    xyz, ts0 = f32(g["mid/xyz"]), g["mid/ts"]
    start = int(g["mid/frame_start"])
    imu = [mc.IMUData(int(t), *map(float, gy), 0.0, 0.0, 0.0) for t, gy in zip(g["mid/imu_ts"], g["mid/imu_gyro"])]
    pts = [mc.LiDARPoint(*map(float, p), 0, int(t), 0, 0) for p, t in zip(xyz, ts0)]
    comp = mc.MotionCompensator({}, context=gpu_ctx)
    for k in range(3):
        if k:
            for s in imu[1:-1]:
                s.gyro_x, s.gyro_z = s.gyro_x + 0.3 * k, s.gyro_z - 0.5 * k
        ts, gyro = mc.imu_to_arrays(imu)
        got = np.array([[p.x, p.y, p.z] for p in comp.compensate_point_cloud(pts, imu, start, 100_000_000)])
        ref = R.compensate_arrays(xyz, ts0, start, ts, gyro)
        assert_scaled_close(got, ref, scale_of(xyz), what=f"edit {k}")
    other = mc.MotionCompensator({}, context=gpu_ctx)
    imu2 = [mc.IMUData(int(t), *map(float, gy), 0.0, 0.0, 0.0) for t, gy in zip(g["mid/imu_ts"], g["mid/imu_gyro"])]
    got = np.array([[p.x, p.y, p.z] for p in other.compensate_point_cloud(pts, imu2, start, 100_000_000)])
    assert_scaled_close(got, R.compensate_arrays(xyz, ts0, start, *mc.imu_to_arrays(imu2)), scale_of(xyz))
    got = np.array([[p.x, p.y, p.z] for p in comp.compensate_point_cloud(pts, imu, start, 100_000_000)])
    assert_scaled_close(got, R.compensate_arrays(xyz, ts0, start, *mc.imu_to_arrays(imu)), scale_of(xyz))


@pytest.mark.parametrize("rate", [0.5, 2.0, 2.4, 7.7, 8.5, 30.0])
def test_imu_polynomial_tiers_and_thresholds(mc, gpu_ctx, rate):
    """Each wave evaluates sin / cos at the polynomial tier that covers its angles (|theta| <= 1/16,
    <= 1/4, any angle with range reduction): constant rates that put theta = rate * dt on either
    side of the tier bounds within one 0.1 s frame (time-sorted points, so whole waves land on each
    side), plus points before the frame start and a rate change between IMU samples; strict parity
    with the oracle."""
    rng = np.random.default_rng(int(rate * 10))
    ts = np.arange(0, 2_000_000_000, 5_000_000, dtype=np.int64)
    gyro = np.tile(np.array([rate, -0.6 * rate, 0.9 * rate]), (len(ts), 1))
    gyro[len(ts) // 2 + 3:] *= -1.0                      # rate flip inside the frame window
    n = 50_000
    xyz = f32(rng.uniform(-90, 90, (n, 3)))
    start = 1_000_000_000
    t_abs = np.sort(start + rng.integers(-2_000_000, 100_000_000, n))
    comp = mc.MotionCompensator({}, context=gpu_ctx)
    gpu_ctx.set_imu(ts, gyro)
    got = _batch_deskew(gpu_ctx, [xyz], [t_abs - start], "imu", starts=[start])[0][:, :3]
    ref = R.compensate_arrays(xyz, t_abs, start, ts, gyro)
    assert_scaled_close(got, ref, scale_of(xyz), what=f"rate {rate}")
    assert_scaled_close(comp.compensate_arrays(xyz, t_abs, start, ts, gyro), ref, scale_of(xyz), what="float64 rows")


def test_imu_slow_path_wide_subtile(mc, gpu_ctx):
    """1024 points spread over 1.5 s at 200 Hz IMU -> ~300 segments in one sub-tile."""
    rng = np.random.default_rng(4)
    ts = np.arange(0, 4_000_000_000, 5_000_000, dtype=np.int64)
    gyro = rng.normal(0, 2.0, (len(ts), 3))
    n = 3000
    xyz = f32(rng.uniform(-80, 80, (n, 3)))
    start = 1_000_000_000
    t_abs = start + rng.integers(-500_000_000, 1_000_000_000, n)
    comp = mc.MotionCompensator({}, context=gpu_ctx)
    gpu_ctx.set_imu(ts, gyro)
    got = _batch_deskew(gpu_ctx, [xyz], [t_abs - start], "imu", starts=[start])[0][:, :3]
    ref = R.compensate_arrays(xyz, t_abs, start, ts, gyro)
    assert_scaled_close(got, ref, scale_of(xyz))
    assert_scaled_close(comp.compensate_arrays(xyz, t_abs, start, ts, gyro), ref, scale_of(xyz), what="float64 rows")


# ---------------------------------------------------------------------------------------------
# timing hooks and single-rank RCCL gather
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("mode", ["pose_slerp", "imu", "frame"])
def test_timing_counts_launches(mc, gpu_ctx, mode):
    b, tr, times = _c2_batch(mc, gpu_ctx, frames=8, n=10_000)
    b.set_frame_starts((times * 1e9).astype(np.int64))
    gpu_ctx.set_imu(*mc.trajectory.imu_from_trajectory(tr, 200.0))
    out = gpu_ctx.batch(b.counts)
    gpu_ctx.read_timing()
    gpu_ctx.timing(True)
    for _ in range(3):
        gpu_ctx.deskew(b, out, mode=mode)
    t = gpu_ctx.read_timing()
    gpu_ctx.timing(False)
    # calls 1 and 2 run k_prep; call 2's launch also prepares call 3's tables (identical key), so
    # call 3 needs none (mc_deskew's per-call speculation, test_gpu_steps.py).  A build without the
    # fused SLERP kernel (MC_FUSE_SLERP=0) issues the SLERP prep before the plain kernel on every call
    assert t["main_launches"] == 3 and t["main_ms"] > 0
    assert t["prep_launches"] == 2 or (mode == "pose_slerp" and t["prep_launches"] == 3), t


def test_rccl_gather_single_rank(mc, gpu_ctx):
    dist = mc.dist
    rdv = dist.Rendezvous(0, 1)
    comm = dist.RcclComm(gpu_ctx, rdv)
    try:
        b = gpu_ctx.batch([5, 1000, 3])
        b.synth(seed=1, frame_id_base=0)
        merged = dist.gather_merged(gpu_ctx, comm, rdv, b)
        assert np.array_equal(merged.download_aos(), b.download_aos())
        assert comm.allreduce_max([1.5, -2.0]).tolist() == [1.5, -2.0]
        # a shard carrying t_ns (5 columns per block) into a 4-column merged batch: re-pitched copy
        bt = gpu_ctx.batch([300, 0, 70_000, 1], with_time=True)
        bt.synth(seed=3, frame_id_base=0)
        merged = dist.gather_merged(gpu_ctx, comm, rdv, bt)
        assert not merged.with_time
        assert np.array_equal(merged.download_aos(), bt.download_aos())
    finally:
        comm.close()


# ---------------------------------------------------------------------------------------------
# device stager: (N,4) f64 AoS <-> f32 SoA columns inside HBM
# ---------------------------------------------------------------------------------------------
def test_device_stager_roundtrip(mc, gpu_ctx):
    counts = np.array([100_000, 3, 0, 7, 20_001, 2049])
    b = gpu_ctx.batch(counts)
    b.synth(seed=2, frame_id_base=0)
    buf = gpu_ctx.device_buffer(b.n_points * 32)
    b.fetch_aos_device(buf)
    aos = buf.to_host(np.float64, (b.n_points, 4))
    assert np.array_equal(aos, b.download_aos())
    hx, hy, hz, hi, _ = synth.synth_batch(counts, seed=2, frame_id_base=0)
    assert np.array_equal(aos, np.stack([hx, hy, hz, hi], 1).astype(np.float64))
    b2 = gpu_ctx.batch(counts)
    b2.stage_aos_device(buf)
    for c1, c2 in zip(b.download_columns(), b2.download_columns()):
        assert np.array_equal(c1, c2)
    # wider rows (ld = 6, the reference passes extra columns through points[:, :3] / [:, 3])
    wide = np.concatenate([aos, np.full((len(aos), 2), 7.0)], axis=1)
    buf6 = gpu_ctx.device_buffer(wide.nbytes)
    buf6.from_host(wide)
    b3 = gpu_ctx.batch(counts)
    b3.stage_aos_device(buf6, ld=6)
    assert np.array_equal(b3.download_aos(), aos)
    with pytest.raises(IndexError):
        b3.stage_aos_device(buf6, ld=3)


def test_host_array_paths_zero_copy_and_pipeline(mc, gpu_ctx):
    """transform_pointcloud / align_frames / run_alignment on host arrays: the zero-copy kernels
    below 32k rows and the chunked DMA pipeline above (1M-row chunks), ragged frames, empty
    frames, wider rows, float64 results against the oracle."""
    rng = np.random.default_rng(12)
    sim = mc.LiDARMotionSimulator(dict(CFGS["urban_complex"]), context=gpu_ctx)
    for n in (5, 40_000, 1_300_000):
        pts = np.column_stack([rng.normal(0, 50, (n, 3)), rng.uniform(0, 1, n), rng.normal(0, 1, n)])
        pose = {"translation": rng.normal(0, 500, 3), "rotation": rng.uniform(-np.pi, np.pi, 3)}
        out = sim.transform_pointcloud(pts, pose)
        ref = R.transform_pointcloud(pts, pose)
        np.testing.assert_allclose(out, ref, rtol=0, atol=1e-9 * (1 + np.abs(ref).max()))
        assert np.array_equal(out[:, 3], pts[:, 3])
    tr = traj_of("urban_complex")
    sizes = [0, 17, 300_000, 0, 1_100_001, 5, 900_000, 64]
    scans = [np.column_stack([rng.normal(0, 40, (m, 3)), rng.uniform(0, 1, m)] +
                             ([rng.normal(0, 1, (m, 2))] if i % 3 == 1 else [])) for i, m in enumerate(sizes)]
    times = np.linspace(0, 119.9, len(sizes))
    got = sim.run_alignment(scans, tr, times)
    ref = R.align_frames(scans, tr, times)
    for g, r, s in zip(got, ref, scans):
        assert g.shape == r.shape
        if len(r):
            np.testing.assert_allclose(g, r, rtol=0, atol=1e-9 * (1 + np.abs(r).max()))
            assert np.array_equal(g[:, 3], s[:, 3])
    small = [s[:50] for s in scans]
    poses = [{"translation": rng.normal(0, 100, 3), "rotation": rng.uniform(-1, 1, 3)} for _ in small]
    for g, s, p in zip(sim.align_frames(small, poses), small, poses):
        np.testing.assert_allclose(g, R.transform_pointcloud(s, p), rtol=0, atol=1e-9)


@pytest.mark.parametrize("mode", ["pose_slerp", "frame"])
def test_launch_spans_match_events(mc, gpu_ctx, mode):
    """mc_timing_read_spans: every timed deskew launch's own workgroup span (the bench line's
    roofline kernel time) is positive and within its HIP-event time, which also holds the dispatch
    gap ahead of the launch; untimed launches take no span."""
    counts = np.full(64, 100_000, np.int64)
    b_in = gpu_ctx.batch(counts, with_time=mode != "frame")
    b_out = gpu_ctx.batch(counts)
    b_in.synth(seed=5, frame_id_base=0)
    times = np.arange(64) * 0.1 + 1.0
    b_in.set_frame_times(times)
    sim = mc.LiDARMotionSimulator({"duration": 60.0, "trajectory_type": "figure_eight", "lidar_fps": 10})
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    gpu_ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    gpu_ctx.read_timing_each()
    gpu_ctx.read_timing_spans()
    gpu_ctx.deskew_steps(b_in, b_out, 9, mode=mode, sample_every=3)
    gpu_ctx.sync()
    each = gpu_ctx.read_timing_each()
    spans = gpu_ctx.read_timing_spans()
    assert len(each) == 3 and len(spans) == 3
    for e, s in zip(each, spans):
        assert 0.0 < s <= e * 1e3 + 0.5, (s, e)
    gpu_ctx.timing(False)
    gpu_ctx.deskew(b_in, b_out, mode=mode)          # untimed
    gpu_ctx.sync()
    assert gpu_ctx.read_timing_spans() == []
    gpu_ctx.read_timing()


@pytest.mark.gpu
def test_local_rank_wraps_to_the_visible_devices(mc, monkeypatch):
    """Context() under a launcher's LOCAL_RANK picks LOCAL_RANK modulo the visible devices (a rank
    given its own HIP_VISIBLE_DEVICES sees one device); an explicit device is taken as given."""
    n = mc.Context.device_count()
    monkeypatch.delenv("MCDESKEW_DEVICE", raising=False)
    monkeypatch.setenv("LOCAL_RANK", str(n + 1))
    ctx = mc.Context()
    assert ctx.device == (n + 1) % n
    b = ctx.batch([300])
    b.synth(seed=1)
    assert b.download_aos().shape == (300, 4)
    b.close()
    monkeypatch.setenv("MCDESKEW_DEVICE", str(n + 1))
    with pytest.raises(ValueError, match="out of range"):
        mc.Context()


@pytest.mark.gpu
def test_set_imu_uploads_on_any_byte_change(mc, gpu_ctx):
    """Context.set_imu skips the upload only for the very bytes the device holds: a gyro sample
    turned from 0.0 into -0.0 (equal as numbers) is uploaded again, as Context.set_environment does
    for scenes."""
    ts = np.arange(10, dtype=np.int64) * 5_000_000
    g = np.zeros((10, 3))
    gpu_ctx.set_imu(ts, g)
    first = gpu_ctx._imu_last
    gpu_ctx.set_imu(ts.copy(), g.copy())
    assert gpu_ctx._imu_last is first
    g2 = g.copy()
    g2[3, 1] = -0.0
    gpu_ctx.set_imu(ts, g2)
    assert gpu_ctx._imu_last is not first and np.signbit(gpu_ctx._imu_last[1][3, 1])
