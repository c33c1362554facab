"""Randomised parity sweep (fixed seeds): ragged batches of random frame sizes, point times drawn
from several regimes (sorted within the frame, shuffled, spanning seconds, before the frame start),
random pose tables (sparse / dense / single pose, yaw wrapping) and IMU streams (quiet / spiky),
every mode, through the C-ABI, against the oracle at the parity bar.  Each case exercises a
different mix of the kernels' paths (SGPR records, per-sub-tile windows, LDS windows, out-of-line
search; f32 and f64 IMU angles)."""
import numpy as np
import pytest

from conftest import assert_scaled_close, scale_of
from oracle import restatement as R

pytestmark = pytest.mark.gpu


def _case(seed):
    rng = np.random.default_rng(seed)
    F = int(rng.integers(1, 24))
    counts = rng.choice([0, 1, 3, 4, 255, 256, 257, 1023, 1024, 1025, 4096, 20_000], F)
    kinds = rng.integers(0, 4, F)
    t_ns = []
    for n, k in zip(counts, kinds):
        if k == 0:
            t = np.sort(rng.integers(0, 100_000_000, n))                 # a Mid-70 frame
        elif k == 1:
            t = rng.integers(0, 100_000_000, n)                          # shuffled
        elif k == 2:
            t = rng.integers(-1_500_000_000, 1_500_000_000, n)            # seconds either side
        else:
            t = np.sort(rng.integers(-3_000_000, 3_000_000, n))          # around the frame start
        t_ns.append(t.astype(np.int64))
    pts = [np.column_stack([rng.uniform(-90, 90, (n, 3)), rng.uniform(0, 1, n)]) for n in counts]
    T = int(rng.choice([1, 2, 7, 300, 4000]))
    dur = float(rng.choice([30.0, 120.0]))
    time = np.linspace(0, dur, T) if T > 1 else np.array([0.0])
    yaw = np.cumsum(rng.normal(0, 0.3, T))
    rpy = np.column_stack([rng.normal(0, 0.05, T), rng.normal(0, 0.05, T),
                           (yaw + np.pi) % (2 * np.pi) - np.pi])                # wraps at +-pi
    pos = np.cumsum(rng.normal(0, 2.0, (T, 3)), axis=0)
    tr = {"time": time, "position_gps": pos, "orientation_imu": rpy}
    times = np.sort(rng.uniform(-1.0, dur + 1.0, F))
    M = int(rng.choice([1, 50, 4000]))
    imu_ts = np.sort(rng.integers(-2_000_000_000, int((dur + 2) * 1e9), M)).astype(np.int64)
    gyro = rng.normal(0, float(rng.choice([0.2, 5.0])), (M, 3))
    if M > 10:
        gyro[rng.integers(0, M, 3)] *= 200.0                                     # yaw-wrap spikes
    return counts, pts, t_ns, tr, times, imu_ts, gyro


@pytest.mark.parametrize("seed", range(40))
def test_random_batches_all_modes(mc, gpu_ctx, seed):
    counts, pts, t_ns, tr, times, imu_ts, gyro = _case(seed)
    n = int(counts.sum())
    aos = np.concatenate(pts) if n else np.zeros((0, 4))
    tt = np.concatenate(t_ns) if n else np.zeros(0, np.int64)
    starts = np.round(times * 1e9).astype(np.int64)
    b = gpu_ctx.batch(counts, with_time=True)
    try:
        if n:
            b.upload_aos(aos)
            b.upload_time(tt.astype(np.int32))
        b.set_frame_times(times)
        b.set_frame_starts(starts)
        gpu_ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
        gpu_ctx.set_imu(imu_ts, gyro)
        offs = np.concatenate([[0], np.cumsum(counts)])
        idx = R.select_pose_index(tr["time"], times)
        for mode in ("frame", "pose_slerp", "imu"):
            out = gpu_ctx.deskew(b, mode=mode)
            got = out.download_aos()
            out.close()
            assert np.array_equal(got[:, 3], aos[:, 3].astype(np.float32).astype(np.float64))
            for f in range(len(counts)):
                s = slice(offs[f], offs[f + 1])
                if counts[f] == 0:
                    continue
                p = aos[s, :3].astype(np.float32).astype(np.float64)    # the batch holds float32
                if mode == "frame":
                    k = idx[f]
                    ref = R.transform_pointcloud(np.column_stack([p, aos[s, 3]]),
                                                 {"translation": tr["position_gps"][k],
                                                  "rotation": tr["orientation_imu"][k]})[:, :3]
                    sc = scale_of(p, tr["position_gps"][k])
                elif mode == "pose_slerp":
                    Rm, pp = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"],
                                          times[f] + tt[s] * 1e-9)
                    ref = np.einsum("nij,nj->ni", Rm, p) + pp
                    sc = scale_of(p, pp)
                else:
                    ref = R.compensate_arrays(p, starts[f] + tt[s], starts[f], imu_ts, gyro)
                    sc = scale_of(p)
                assert_scaled_close(got[s, :3], ref, sc, what=f"seed {seed} {mode} frame {f} ({counts[f]} pts)")
    finally:
        b.close()


@pytest.mark.parametrize("seed", range(8))
def test_random_codec_frames(mc, gpu_ctx, seed):
    """LVX and ASCII PCD of random ragged frames against the oracle, byte for byte: magnitudes from
    1e-9 to 1e9 (packed and byte-path PCD lines mixed within tiles), float32-valued and exact-tie
    values, -0.0 and inf in the PCD case (LVX rejects non-finite values like the reference)."""
    from oracle import codecs as C

    rng = np.random.default_rng(100 + seed)
    F = int(rng.integers(1, 12))
    counts = rng.choice([0, 1, 95, 96, 97, 255, 256, 257, 1000, 5000], F)
    frames = []
    for n in counts:
        mag = 10.0 ** rng.uniform(-9, rng.choice([3.5, 9.0]), (n, 4))
        v = rng.choice([-1.0, 1.0], (n, 4)) * mag
        v[:, 3] = np.abs(v[:, 3]) % 1.2
        if n > 10:
            v[::5, 0] = np.round(v[::5, 0] * 128) / 128                          # exact %.6f ties
            v[1::7, 1] = v[1::7, 1].astype(np.float32)
            v[2::11, 2] = -0.0
        frames.append(v)
    pcds = mc.codecs.encode_pcd_frames(frames, gpu_ctx)
    special = [f.copy() for f in frames]
    for f in special:
        if len(f) > 3:
            f[3, 0] = np.inf
    assert all(p == C.pcd_ascii_bytes(f) for p, f in zip(pcds, frames))
    assert all(p == C.pcd_ascii_bytes(f) for p, f in zip(mc.codecs.encode_pcd_frames(special, gpu_ctx), special))
    lvx_frames = [{"frame_id": 3 * i + 1, "timestamp": 0.05 * i + 1e-3, "points": np.clip(f, -2e6, 2e6)}
                  for i, f in enumerate(frames)]
    assert mc.codecs.encode_lvx(lvx_frames, gpu_ctx) == C.lvx_bytes(lvx_frames)
