"""GPU: n deskew steps (mc_deskew_steps: each step's launch also runs the next step's prep) give the
plain calls' bytes.

Every step recomputes its pose prep and reruns its kernel, so after any number of steps the output
is bit-identical to one mc_deskew call on the same batch; the oracle check of that output is the
parity tests' (test_gpu_parity.py).  Here: byte equality with mc_deskew over every mode, ragged
batches, odd / even step counts, interleaving with plain calls, new tables between calls, and the
sampled timing events.
"""
import numpy as np
import pytest

from conftest import assert_scaled_close, scale_of
from oracle import restatement as R
from oracle import synth

pytestmark = pytest.mark.gpu

CFG = {"duration": 120.0, "trajectory_type": "figure_eight", "environment_complexity": "complex",
       "max_speed": 12.0, "lidar_fps": 10}


def _setup(mc, ctx, counts, seed=3):
    sim = mc.LiDARMotionSimulator(dict(CFG), context=ctx)
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[: len(counts)]
    b = ctx.batch(np.asarray(counts), with_time=True)
    b.synth(seed=seed, frame_id_base=1000)
    b.set_frame_times(times)
    b.set_frame_starts((times * 1e9).astype(np.int64))
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    ts, gyro = mc.trajectory.imu_from_trajectory(tr, 200.0)
    ctx.set_imu(ts, gyro)
    return b, tr, times


def _cols(b):
    return np.stack(b.download_columns())


@pytest.mark.parametrize("mode", ["frame", "pose_slerp", "imu"])
@pytest.mark.parametrize("n_steps", [1, 2, 7])
def test_steps_match_plain_calls(mc, gpu_ctx, mode, n_steps):
    counts = [3000, 0, 1, 257, 20_000, 1023, 4097]
    b, tr, times = _setup(mc, gpu_ctx, counts)
    ref = gpu_ctx.batch(b.counts)
    gpu_ctx.deskew(b, ref, mode=mode)
    want = _cols(ref)
    out = gpu_ctx.batch(b.counts)
    gpu_ctx.deskew_steps(b, out, n_steps, mode=mode)
    gpu_ctx.sync()
    assert np.array_equal(_cols(out), want)
    # again, then interleaved with plain calls on the same tables
    out2 = gpu_ctx.batch(b.counts)
    gpu_ctx.deskew(b, out2, mode=mode)
    gpu_ctx.deskew_steps(b, out, n_steps, mode=mode)
    gpu_ctx.deskew(b, out2, mode=mode)
    gpu_ctx.deskew_steps(b, out, n_steps, mode=mode)
    gpu_ctx.sync()
    assert np.array_equal(_cols(out), want)
    assert np.array_equal(_cols(out2), want)
    for x in (out, out2, ref, b):
        x.close()


def test_steps_oracle_after_new_trajectory(mc, gpu_ctx):
    """Steps after the trajectory grows (new table pointers and sizes): every step's prep reads the
    tables current when it runs (nothing carried over from the last call); checked against the oracle."""
    counts = [5000, 5000, 5000]
    b, tr, times = _setup(mc, gpu_ctx, counts, seed=11)
    out = gpu_ctx.batch(b.counts)
    gpu_ctx.deskew_steps(b, out, 4, mode="pose_slerp")
    gpu_ctx.sync()
    first = _cols(out)
    # a longer, shifted trajectory: every point's pose changes
    T = len(tr["time"]) * 2
    t2 = np.linspace(0.0, tr["time"][-1], T)
    pos2 = np.column_stack([np.interp(t2, tr["time"], tr["position_gps"][:, i]) + 3.0 for i in range(3)])
    rpy2 = np.column_stack([np.interp(t2, tr["time"], tr["orientation_imu"][:, i]) for i in range(3)])
    tr2 = {"time": t2, "position_gps": pos2, "orientation_imu": rpy2}
    gpu_ctx.set_trajectory(t2, pos2, rpy2)
    gpu_ctx.deskew_steps(b, out, 4, mode="pose_slerp")
    gpu_ctx.sync()
    got = _cols(out)
    assert not np.array_equal(got, first)
    hx, hy, hz, hi, ht = synth.synth_batch(b.counts, seed=11, frame_id_base=1000)
    off = 0
    for f, n in enumerate(counts):
        s = slice(off, off + n)
        off += n
        p = np.stack([hx[s], hy[s], hz[s]], axis=1).astype(np.float64)
        ref = R.deskew_pose_slerp(p, ht[s], times[f], tr2)
        _, pos = R.slerp_pose(t2, pos2, rpy2, times[f] + ht[s] * 1e-9)
        assert_scaled_close(got[:3, s].T, ref, scale_of(p, pos), what=f"frame {f}")
    assert np.array_equal(got[3], hi)
    out.close()
    b.close()


@pytest.mark.parametrize("mode", ["frame", "pose_slerp", "imu"])
def test_pipelined_steps_in_place_and_new_frame_times(mc, gpu_ctx, mode):
    """In place (out = in), n pipelined steps compound exactly as n plain calls; new frame times
    between two pipelined calls reach the next call's first step (its prep runs after the upload)."""
    counts = [4000, 17, 0, 9000, 2048]
    b, tr, times = _setup(mc, gpu_ctx, counts, seed=5)
    c = gpu_ctx.batch(b.counts, with_time=True)
    c.synth(seed=5, frame_id_base=1000)
    c.set_frame_times(times)
    c.set_frame_starts((times * 1e9).astype(np.int64))
    for _ in range(3):
        gpu_ctx.deskew(c, c, mode=mode)
    gpu_ctx.deskew_steps(b, b, 3, mode=mode)
    gpu_ctx.sync()
    assert np.array_equal(_cols(b), _cols(c))
    t2 = times + 0.037
    for x in (b, c):
        x.synth(seed=5, frame_id_base=1000)
    out, want = gpu_ctx.batch(b.counts), gpu_ctx.batch(b.counts)
    gpu_ctx.deskew_steps(b, out, 2, mode=mode)
    b.set_frame_times(t2)
    b.set_frame_starts((t2 * 1e9).astype(np.int64))
    gpu_ctx.deskew_steps(b, out, 2, mode=mode)
    gpu_ctx.deskew(b, want, mode=mode)
    gpu_ctx.sync()
    assert np.array_equal(_cols(out), _cols(want))
    for x in (out, want, c, b):
        x.close()


def test_pipelined_steps_sampled_timing(mc, gpu_ctx):
    b, _, _ = _setup(mc, gpu_ctx, [20_000] * 8)
    out = gpu_ctx.batch(b.counts)
    gpu_ctx.read_timing()
    gpu_ctx.deskew_steps(b, out, 20, mode="pose_slerp", sample_every=5)   # steps 2, 7, 12, 17
    t = gpu_ctx.read_timing()
    assert t["main_launches"] == 4 and t["main_ms"] > 0
    gpu_ctx.deskew_steps(b, out, 20, mode="pose_slerp")
    assert gpu_ctx.read_timing()["main_launches"] == 0
    out.close()
    b.close()


def test_steps_argument_errors(mc, gpu_ctx):
    b, _, _ = _setup(mc, gpu_ctx, [100])
    out = gpu_ctx.batch(b.counts)
    with pytest.raises(ValueError):
        gpu_ctx.deskew_steps(b, out, 0, mode="frame")
    with pytest.raises(ValueError):
        gpu_ctx.deskew_steps(b, out, 2, mode="frame", sample_every=-1)
    other = gpu_ctx.batch([5, 5])
    with pytest.raises(ValueError):
        gpu_ctx.deskew_steps(b, other, 2, mode="frame")
    for x in (other, out, b):
        x.close()


# ---------------------------------------------------------------------------------------------
# per-call speculation (mc_deskew): a repeated call finds its tables prepared by the previous launch
# ---------------------------------------------------------------------------------------------
def _fresh(mc, counts, mode, setup):
    """The reference bytes: the same call on a fresh context (no speculation history)."""
    ctx = mc.Context(0)
    b, tr, times = _setup(mc, ctx, counts)
    setup(ctx, b)
    out = ctx.deskew(b, ctx.batch(b.counts), mode=mode)
    return _cols(out)


@pytest.mark.parametrize("mode", ["frame", "pose_slerp", "imu"])
def test_repeated_calls_speculate_and_every_input_change_misses(mc, gpu_ctx, mode):
    """Identical calls after the first skip their k_prep (the previous launch prepared the tables);
    any change to a prep input between calls — trajectory, IMU table, frame times, frame starts, t_ns,
    another batch in between, a step sequence in between — must give the bytes of a fresh call."""
    counts = [3000, 0, 1, 257, 20_000, 1023, 4097]
    ctx = gpu_ctx
    b, tr, times = _setup(mc, ctx, counts)
    out = ctx.batch(b.counts)
    ref = _fresh(mc, counts, mode, lambda c, bb: None)
    ctx.read_timing()
    ctx.timing(True)
    for _ in range(5):
        ctx.deskew(b, out, mode=mode)
        assert np.array_equal(_cols(out), ref)
    t = ctx.read_timing()
    ctx.timing(False)
    assert t["main_launches"] == 5
    # calls 1 and 2 prepare; 3.. find the tables ready.  A build without the fused SLERP kernel
    # (MC_FUSE_SLERP=0) prepares every SLERP call
    assert t["prep_launches"] == 2 or (mode == "pose_slerp" and t["prep_launches"] == 5), t
    rng = np.random.default_rng(5)
    tr2 = {k: v.copy() for k, v in tr.items()}
    tr2["orientation_imu"] = tr2["orientation_imu"] + rng.normal(0, 0.05, tr2["orientation_imu"].shape)
    tr2["position_gps"] = tr2["position_gps"] + 1.5
    ts, gyro = mc.trajectory.imu_from_trajectory(tr, 200.0)
    t_new = rng.integers(0, 100_000_000, int(np.sum(counts))).astype(np.int32)
    changes = [
        ("trajectory", lambda c, bb: c.set_trajectory(tr2["time"], tr2["position_gps"], tr2["orientation_imu"])),
        ("imu", lambda c, bb: c.set_imu(ts, gyro * 1.7)),
        ("frame_times", lambda c, bb: bb.set_frame_times(times + 0.013)),
        ("frame_starts", lambda c, bb: bb.set_frame_starts((times * 1e9).astype(np.int64) + 7_000_000)),
        ("t_ns", lambda c, bb: bb.upload_time(t_new)),
    ]
    applied = []
    for name, fn in changes:
        fn(ctx, b)
        applied.append(fn)
        want = _fresh(mc, counts, mode, lambda c, bb, fs=tuple(applied): [f(c, bb) for f in fs])
        for _ in range(3):   # the miss, then speculation on the new inputs
            ctx.deskew(b, out, mode=mode)
            assert np.array_equal(_cols(out), want), name
    # another batch in between (its own key), then back; a pipelined step sequence in between
    other = ctx.batch(np.asarray([500, 7]), with_time=True)
    other.synth(seed=9, frame_id_base=0)
    other.set_frame_times(times[:2])
    other.set_frame_starts((times[:2] * 1e9).astype(np.int64))
    o2 = ctx.batch(other.counts)
    for k in range(6):
        ctx.deskew(other if k % 2 else b, o2 if k % 2 else out, mode=mode)
    ctx.deskew_steps(b, out, 3, mode=mode)
    ctx.deskew(b, out, mode=mode)
    assert np.array_equal(_cols(out), want)


# ---------------------------------------------------------------------------------------------
# device-measured sub-tile order (mc_tune_order)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("mode", ["frame", "pose_slerp", "imu"])
def test_tune_order_keeps_bytes_and_applies_per_size(mc, gpu_ctx, mode):
    """mc_tune_order times both sub-tile orders and keeps the mode's default order (XCD-contiguous for
    frame, dealt for IMU and small SLERP batches) unless the other is at least 1 % faster, for the
    mode and batch size; the deskew output is the same bytes whichever order runs (every later
    call, incl. pipelined steps), and a batch of another size keeps the default order."""
    counts = [3000, 0, 1, 257, 20_000, 1023, 4097]
    ctx = mc.Context(0)
    b, tr, times = _setup(mc, ctx, counts)
    ref = _fresh(mc, counts, mode, lambda c, bb: None)
    out = ctx.batch(b.counts)
    r = ctx.tune_order(b, out, mode=mode, launches=3, rounds=2)
    assert r["chosen"] in ("dealt", "xcd") and r["dealt_us"] > 0 and r["xcd_us"] > 0, r
    default = "xcd" if mode == "frame" else "dealt"
    other = "dealt" if default == "xcd" else "xcd"
    assert r["chosen"] == (other if r[other + "_us"] < r[default + "_us"] * (1.0 - 0.01) else default), r
    assert np.array_equal(_cols(out), ref)        # the tuning launches wrote the same output
    out2 = ctx.batch(b.counts)
    ctx.deskew(b, out2, mode=mode)
    assert np.array_equal(_cols(out2), ref)
    ctx.deskew_steps(b, out2, 3, mode=mode)
    assert np.array_equal(_cols(out2), ref)
    with pytest.raises(ValueError):               # in place: repeated launches would compound
        ctx.tune_order(b, b, mode=mode)
    empty = ctx.batch([0, 0], with_time=True)
    empty.set_frame_times(times[:2])
    empty.set_frame_starts((times[:2] * 1e9).astype(np.int64))
    assert ctx.tune_order(empty, ctx.batch([0, 0]), mode=mode)["chosen"] is None
