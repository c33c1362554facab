"""GPU: n deskew steps replayed as one HIP graph (mc_deskew_steps) give the plain calls' bytes.

Every step of the graph recomputes its pose prep and reruns its kernel, so after any number of
replays the output is bit-identical to one mc_deskew call on the same batch; the oracle check of
that output is the parity tests' (test_gpu_parity.py).  Here: byte equality with mc_deskew over
every mode, ragged batches, odd / even step counts, interleaving with plain calls, re-capture when
the launch arguments change, and the sampled timing events.
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
    # replay of the cached graph, then interleaved with plain calls on the same tables
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


def test_steps_oracle_and_recapture_on_new_trajectory(mc, gpu_ctx):
    """A graph replayed after the trajectory grows (new table pointers and sizes) must be re-captured:
    the output follows the new table (checked against the oracle), not the old graph's."""
    counts = [5000, 5000, 5000]
    b, tr, times = _setup(mc, gpu_ctx, counts, seed=11)
    out = gpu_ctx.batch(b.counts)
    gpu_ctx.deskew_steps(b, out, 4, mode="pose_slerp", prepare=True)   # capture only
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


def test_steps_sampled_timing(mc, gpu_ctx):
    b, _, _ = _setup(mc, gpu_ctx, [20_000] * 8)
    out = gpu_ctx.batch(b.counts)
    gpu_ctx.read_timing()
    gpu_ctx.deskew_steps(b, out, 20, mode="pose_slerp", sample_every=10)   # steps 5 and 15
    gpu_ctx.deskew_steps(b, out, 20, mode="pose_slerp", sample_every=10)
    t = gpu_ctx.read_timing()
    assert t["main_launches"] == 4 and t["prep_launches"] == 4
    assert t["main_ms"] > 0 and t["prep_ms"] > 0
    assert gpu_ctx.read_timing()["main_launches"] == 0
    # without sampling nothing is recorded
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
