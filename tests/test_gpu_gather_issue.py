"""GPU: the merged-cloud gather's plan / staging / re-pitch on the device, the step-issue protocol
(per-step prep as an any-order packet on the kernel's queue), t_ns span invalidation, and BASELINE
config 5's whole job on one device (past 2^32 input values).

The multi-rank RCCL gather cannot run on a one-GPU box (RCCL refuses two ranks on one device), so
``mc_gather_batches`` merges n shard batches in one process through the same plan, staging and
re-pitch code as ``mc_comm_gather_batch`` (comm.cpp), device copies standing in for the receives.
"""
import numpy as np
import pytest

from conftest import assert_scaled_close, scale_of
from oracle import restatement as R
from oracle import synth

pytestmark = pytest.mark.gpu

URBAN = {"duration": 120.0, "trajectory_type": "figure_eight", "environment_complexity": "complex",
         "max_speed": 12.0, "lidar_fps": 10}


# ---------------------------------------------------------------------------------------------
# the merged-cloud gather (LMC:887-889)
# ---------------------------------------------------------------------------------------------
def _shard(ctx, counts, with_time, base):
    b = ctx.batch(np.asarray(counts, np.int64), with_time=with_time)
    b.synth(seed=3, frame_id_base=base)
    return b


@pytest.mark.parametrize("merged_time", [False, True])
def test_gather_batches_equals_vstack(mc, gpu_ctx, merged_time):
    """Ragged shards (empty shard, empty frames, 1..7-point frames, 100 003 points), 4- and
    5-column shards into a 4-column merged batch (staged + re-pitched) or 5-column shards into a
    5-column one, every root: merged == np.vstack of the shards, bit for bit (t_ns too)."""
    rng = np.random.default_rng(11)
    shapes = [[1, 7, 0, 300], [], [100_003], [0, 0], [2048, 2049, 5], [256] * 9]
    for trial in range(4):
        order = rng.permutation(len(shapes))
        counts = [shapes[k] for k in order]
        wt = [True if merged_time else bool(rng.integers(0, 2)) for _ in counts]
        shards = [_shard(gpu_ctx, c, w, 100 * q) for q, (c, w) in enumerate(zip(counts, wt))]
        for root in sorted({0, len(shards) - 1, int(rng.integers(0, len(shards)))}):
            merged = gpu_ctx.batch(np.concatenate([np.asarray(c, np.int64) for c in counts]), with_time=merged_time)
            mc.dist.gather_batches(gpu_ctx, shards, root=root, merged=merged)
            want = np.vstack([s.download_aos() for s in shards])
            assert np.array_equal(merged.download_aos(), want), (trial, root)
            if merged_time:
                assert np.array_equal(merged.download_time(), np.concatenate([s.download_time() for s in shards]))
            merged.close()
        for s in shards:
            s.close()


def test_gather_batches_rejects_narrow_shard(mc, gpu_ctx):
    a = _shard(gpu_ctx, [300], False, 0)
    b = _shard(gpu_ctx, [10], True, 1)
    merged = gpu_ctx.batch([300, 10], with_time=True)
    with pytest.raises(ValueError, match="columns"):
        mc.dist.gather_batches(gpu_ctx, [a, b], merged=merged)


def test_gather_of_deskewed_shards_equals_frame_ordered_vstack(mc, gpu_ctx):
    """The bench's multi-GPU path on one device: a run's frames split by plan_shards into 3 shard
    batches, each deskewed (SLERP) on its own, merged — equals the whole run deskewed as one batch,
    and sampled frames match the oracle (LMC:802-832 + 887-889)."""
    sim = mc.LiDARMotionSimulator(dict(URBAN), context=gpu_ctx)
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:40]
    counts = np.array([(997 * (f + 3)) % 40_000 + 1 for f in range(40)], np.int64)
    gpu_ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    whole = gpu_ctx.batch(counts, with_time=True)
    whole.synth(seed=0, frame_id_base=1000)
    whole.set_frame_times(times)
    ref = gpu_ctx.deskew(whole, gpu_ctx.batch(counts), mode="pose_slerp").download_aos()
    bnd = mc.dist.plan_shards(counts, 3)
    outs = []
    for r in range(3):
        lo, hi = int(bnd[r]), int(bnd[r + 1])
        b = gpu_ctx.batch(counts[lo:hi], with_time=True)
        b.synth(seed=0, frame_id_base=1000 + lo)
        b.set_frame_times(times[lo:hi])
        outs.append(gpu_ctx.deskew(b, gpu_ctx.batch(counts[lo:hi]), mode="pose_slerp"))
    merged = mc.dist.gather_batches(gpu_ctx, outs, root=1)
    got = merged.download_aos()
    assert np.array_equal(got, ref)
    offs = np.concatenate([[0], np.cumsum(counts)])
    for f in (0, int(bnd[1]), 39):
        x, y, z, _, t = synth.synth_frame(int(counts[f]), 0, 1000 + f)
        p = np.stack([x, y, z], 1).astype(np.float64)
        _, pos = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"], times[f] + t * 1e-9)
        assert_scaled_close(got[offs[f]:offs[f + 1], :3], R.deskew_pose_slerp(p, t, times[f], tr), scale_of(p, pos),
                            what=f"frame {f}")
        np.testing.assert_array_equal(merged.download_frames(f, f + 1), got[offs[f]:offs[f + 1]])


# ---------------------------------------------------------------------------------------------
# step issue: any-order prep packets, double-buffered halves, fences
# ---------------------------------------------------------------------------------------------
def _dense_traj(seed, T=3000, dt=0.01):
    rng = np.random.default_rng(seed)
    time = np.arange(T) * dt
    rpy = np.cumsum(rng.normal(0, 0.02, (T, 3)), axis=0)
    pos = np.cumsum(rng.normal(0, 0.05, (T, 3)), axis=0)
    return {"time": time, "position_gps": pos, "orientation_imu": rpy}


def test_output_reused_as_input_recomputes_time_spans(mc, gpu_ctx):
    """a per-point deskew that carries t_ns into another batch rewrites that batch's time
    column, so its cached [min, max] spans must be recomputed before it is used as an input.
    A (t1) -> B -> C, then A (t2, a different 20 ms of each frame) -> B -> C: C matches the oracle
    applied twice both times (a stale span would apply t1's pose segment to t2's points)."""
    tr = _dense_traj(5)                                # 100 Hz poses: 10 ms segments
    gpu_ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    counts = np.array([5000, 3000, 7000], np.int64)
    times = np.array([1.0, 2.05, 7.3])
    A, B, C = (gpu_ctx.batch(counts, with_time=True) for _ in range(3))
    for b in (A, B, C):
        b.set_frame_times(times)
    x, y, z, i, _ = synth.synth_batch(counts, seed=1, frame_id_base=0)
    A.upload_columns(x, y, z, i)
    p = np.stack([x, y, z], 1).astype(np.float64)
    offs = np.concatenate([[0], np.cumsum(counts)])
    rng = np.random.default_rng(2)
    for lo_ms in (0, 75):
        t = np.sort(rng.integers(lo_ms * 1_000_000, (lo_ms + 20) * 1_000_000, int(counts.sum()))).astype(np.int32)
        A.upload_time(t)
        gpu_ctx.deskew(A, B, mode="pose_slerp")
        gpu_ctx.deskew(B, C, mode="pose_slerp")
        got = C.download_aos()[:, :3]
        mid = B.download_aos()[:, :3]        # the float32 values the second step read
        assert np.array_equal(C.download_time(), t)
        for f in range(3):
            s = slice(offs[f], offs[f + 1])
            once = R.deskew_pose_slerp(p[s], t[s], times[f], tr)
            twice = R.deskew_pose_slerp(mid[s], t[s], times[f], tr)
            _, pos = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"], times[f] + t[s] * 1e-9)
            assert_scaled_close(mid[s], once, scale_of(p[s], pos), what=f"t window {lo_ms} ms frame {f} (B)")
            assert_scaled_close(got[s], twice, scale_of(mid[s], pos), what=f"t window {lo_ms} ms frame {f}")


def test_interleaved_calls_equal_isolated_calls(mc, gpu_ctx):
    """Many calls queued back to back without a sync (each step's prep an any-order packet beside
    the previous kernel, alternating table halves, three batches, all modes, in-place and out of
    place) give the bytes of the same calls each followed by a sync."""
    sim = mc.LiDARMotionSimulator(dict(URBAN), context=gpu_ctx)
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()
    gpu_ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    ts, gyro = mc.trajectory.imu_from_trajectory(tr, 200.0)
    gpu_ctx.set_imu(ts, gyro)
    specs = [(np.full(30, 20_000), 0), (np.array([1, 70_000, 0, 5, 33_333]), 200), (np.full(7, 150_000), 500)]
    ins, xyz = [], []
    for counts, f0 in specs:
        b = gpu_ctx.batch(counts, with_time=True)
        b.synth(seed=4, frame_id_base=f0)
        tf = times[f0:f0 + len(counts)]
        b.set_frame_times(tf)
        b.set_frame_starts((tf * 1e9).astype(np.int64))
        ins.append(b)
        c = gpu_ctx.batch(counts)
        c.synth(seed=4, frame_id_base=f0)
        c.set_frame_times(tf)
        xyz.append(c)
    plan = [(0, "pose_slerp"), (1, "imu"), (2, "frame"), (0, "imu"), (1, "pose_slerp"), (2, "pose_slerp"),
            (0, "frame"), (1, "frame"), (2, "imu"), (0, "pose_slerp")]

    def run(sync_each):
        """Every call of the plan; returns the outputs and, when synced, each call's result."""
        outs = [gpu_ctx.batch(c) for c, _ in specs]
        res = []
        for k, mode in plan:
            gpu_ctx.deskew(xyz[k] if mode == "frame" else ins[k], outs[k], mode=mode)
            if sync_each:
                res.append(outs[k].download_aos())
        return outs, res

    _, iso = run(True)
    outs, _ = run(False)          # all ten calls queued back to back, no sync in between
    for k in range(3):
        last = max(j for j, (kk, _) in enumerate(plan) if kk == k)
        assert np.array_equal(outs[k].download_aos(), iso[last]), k

    # in-place frame-mode steps queued back to back (each reads the previous step's output) vs the
    # same steps with a sync after each, and vs the oracle applied five times
    a, b = xyz[0], gpu_ctx.batch(specs[0][0])
    b.synth(seed=4, frame_id_base=0)
    b.set_frame_times(times[:30])
    before = a.download_aos()
    for _ in range(5):
        gpu_ctx.deskew(a, a, mode="frame")
    for _ in range(5):
        gpu_ctx.deskew(b, b, mode="frame")
        gpu_ctx.sync()
    chained = a.download_aos()
    assert np.array_equal(chained, b.download_aos())
    ref = before[:, :3].copy()
    idx = R.select_pose_index(tr["time"], times[:30])
    offs = np.concatenate([[0], np.cumsum(specs[0][0])])
    for f in range(30):
        s = slice(offs[f], offs[f + 1])
        Rm = R.euler_xyz_matrix(tr["orientation_imu"][idx[f]])
        for _ in range(5):
            ref[s] = ref[s] @ Rm.T + tr["position_gps"][idx[f]]
    # five float32 round trips between the steps: the scaled bar (a coordinate near 0 after one step
    # carries that step's float32 rounding into the next)
    assert_scaled_close(chained[:, :3], ref, 5 * (np.linalg.norm(ref, axis=1) + 100.0), what="5 chained steps",
                        strict=False)


# ---------------------------------------------------------------------------------------------
# BASELINE config 5's whole job on one device
# ---------------------------------------------------------------------------------------------
def test_config5_whole_job_past_2_32_values(mc, gpu_ctx):
    """BASELINE config 5 as stated, on ONE MI355X: 1200 x 1M-point frames (1.2 G points) of the
    urban_complex run (LMC:792-793), 6.0 G values in the 5-column input — past 2^32 — and 4.8 G in
    the 4-column output; SLERP into the output batch, then frame mode in place on it
    (LMC:772-776).  Frames at both ends and on both sides of the 2^32-value boundary of the input
    (and of the output) are checked against the oracle."""
    F, n = 1200, 1_000_000
    sim = mc.LiDARMotionSimulator(dict(URBAN), context=gpu_ctx)
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()
    assert len(times) == F
    b = gpu_ctx.batch(np.full(F, n), with_time=True)
    assert 5 * b.padded_points > 2 ** 32
    b.synth(seed=0, frame_id_base=1000)
    b.set_frame_times(times)
    gpu_ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    out = gpu_ctx.deskew(b, gpu_ctx.batch(b.counts), mode="pose_slerp")
    assert 4 * out.padded_points > 2 ** 32
    b.close()
    edge_in = 2 ** 32 // (5 * n)          # the frame holding input value 2^32
    edge_out = 2 ** 32 // (4 * n)         # the frame holding output value 2^32
    check = sorted({0, 1, edge_in - 1, edge_in, edge_in + 1, edge_out - 1, edge_out, edge_out + 1, F - 2, F - 1})
    slerp = {f: out.download_frames(f, f + 1) for f in check}
    out.set_frame_times(times)
    gpu_ctx.deskew(out, out, mode="frame")
    idx = R.select_pose_index(tr["time"], times)
    for f in check:
        x, y, z, i, t = synth.synth_frame(n, 0, 1000 + f)
        p = np.stack([x, y, z], 1).astype(np.float64)
        g1 = slerp[f]
        assert np.array_equal(g1[:, 3], i.astype(np.float64)), f
        _, pos = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"], times[f] + t * 1e-9)
        assert_scaled_close(g1[:, :3], R.deskew_pose_slerp(p, t, times[f], tr), scale_of(p, pos), what=f"slerp {f}")
        k = idx[f]
        ref2 = R.transform_pointcloud(g1, {"translation": tr["position_gps"][k], "rotation": tr["orientation_imu"][k]})
        assert_scaled_close(out.download_frames(f, f + 1)[:, :3], ref2[:, :3], scale_of(g1[:, :3], tr["position_gps"][k]),
                            what=f"frame {f}")
    out.close()
