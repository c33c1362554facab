"""GPU: results written by the hot kernels' store policies are what later kernels on any XCD read.

The per-point and frame kernels store their output with cache-policy bits (`sc1` write-through,
`nt`; kernels.hpp st_pol); the stagers with `nt`.  MI355X has one L2 per XCD, so a line of the
output buffer that another XCD's L2 still holds from an earlier kernel (a fill, a read) must not
be seen by a later kernel instead of the new data.  Each case: fill the output buffer with other
data (normal stores), read it on every XCD (checksum kernel), overwrite it with the kernel under
test, then compare the device checksum of the result with the checksum of the same result written
into a buffer that no kernel touched before.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _setup(mc, ctx, frames=64, n=100_000):
    sim = mc.LiDARMotionSimulator({"duration": 120.0, "trajectory_type": "figure_eight", "max_speed": 12.0,
                                   "lidar_fps": 10})
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:frames]
    counts = np.full(frames, n, np.int64)
    b_in = ctx.batch(counts, with_time=True)
    b_in.synth(seed=4, frame_id_base=77)
    b_in.set_frame_times(times)
    b_in.set_frame_starts((times * 1e9).astype(np.int64))
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    ts, g = mc.trajectory.imu_from_trajectory(tr, 200.0)
    ctx.set_imu(ts, g)
    return b_in, counts


@pytest.mark.parametrize("mode", ["pose_slerp", "imu", "frame"])
def test_kernel_output_seen_by_later_kernels(mc, gpu_ctx, mode):
    b_in, counts = _setup(mc, gpu_ctx)
    fresh = gpu_ctx.batch(counts)
    gpu_ctx.deskew(b_in, fresh, mode=mode)
    want = fresh.checksum()
    out = gpu_ctx.batch(counts)
    for r in range(4):
        out.synth(seed=100 + r, frame_id_base=5)   # other data, normal stores
        stale = out.checksum()                     # ... read into the L2s
        gpu_ctx.deskew(b_in, out, mode=mode)
        got = out.checksum()
        assert not np.array_equal(stale, want)
        assert np.array_equal(got, want), (mode, r, got, want)
    for x in (out, fresh, b_in):
        x.close()


def test_stager_output_seen_by_later_kernels(mc, gpu_ctx):
    b_in, counts = _setup(mc, gpu_ctx)
    src = gpu_ctx.batch(counts)
    src.synth(seed=8, frame_id_base=3)
    want = src.checksum()
    buf = gpu_ctx.device_buffer(src.n_points * 32)
    src.fetch_aos_device(buf)                      # SoA -> AoS (nt stores)
    out = gpu_ctx.batch(counts)
    for r in range(4):
        out.synth(seed=200 + r, frame_id_base=9)
        out.checksum()
        out.stage_aos_device(buf)                  # AoS -> SoA (nt stores)
        assert np.array_equal(out.checksum()[:4], want[:4]), r
    for x in (out, src, b_in):
        x.close()
