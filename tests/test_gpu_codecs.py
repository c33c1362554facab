"""GPU codecs byte for byte against files the reference itself wrote
(tests/golden/codecs.npz: LVX v1.1 via LivoxLVXWriter.write_compatible_lvx LMC:57-272, ASCII PCD
via save_pcd LMC:932-948) and against the pinned oracle (oracle/codecs.py) on larger inputs."""
import os

import numpy as np
import pytest

from conftest import golden
from oracle import codecs as C

pytestmark = pytest.mark.gpu


def golden_frames(g):
    return [{"frame_id": int(g[f"lvx/{i}/frame_id"]), "timestamp": float(g[f"lvx/{i}/timestamp"]),
             "points": g[f"lvx/{i}/points"]} for i in range(int(g["lvx/n_frames"]))]


def test_lvx_file_matches_reference_bytes(mc, gpu_ctx, tmp_path):
    g = golden("codecs.npz")
    frames = golden_frames(g)
    assert mc.codecs.encode_lvx(frames, gpu_ctx) == g["lvx/bytes"].tobytes()
    w = mc.LivoxLVXWriter(gpu_ctx)
    fn = str(tmp_path / "t.lvx")
    assert w.write_compatible_lvx(fn, frames) is True
    with open(fn, "rb") as f:
        assert f.read() == g["lvx/bytes"].tobytes()


def test_lvx_failures_like_reference(mc, gpu_ctx, tmp_path):
    w = mc.LivoxLVXWriter(gpu_ctx)
    bad = [{"frame_id": 0, "timestamp": 0.0, "points": np.array([[np.nan, 0, 0, 0.5]])}]
    assert w.write_compatible_lvx(str(tmp_path / "b.lvx"), bad) is False
    bad_i = [{"frame_id": 0, "timestamp": 0.0, "points": np.array([[1.0, 0, 0, np.nan]])}]
    assert w.write_compatible_lvx(str(tmp_path / "c.lvx"), bad_i) is False
    neg_ts = [{"frame_id": 0, "timestamp": -1.0, "points": np.zeros((3, 4))}]
    assert w.write_compatible_lvx(str(tmp_path / "d.lvx"), neg_ts) is False
    with pytest.raises(ValueError):
        w.write_compatible_lvx("", [{"frame_id": 0, "timestamp": 0.0, "points": np.zeros((1, 4))}])
    with pytest.raises(ValueError):
        w.write_compatible_lvx(str(tmp_path / "e.lvx"), [])


def test_lvx_large_ragged_vs_oracle(mc, gpu_ctx):
    rng = np.random.default_rng(5)
    frames = []
    for i, n in enumerate([0, 1, 95, 96, 97, 191, 192, 5000, 20011, 0, 3]):
        p = np.column_stack([rng.normal(0, 10 ** rng.uniform(-3, 7), (n, 3)), rng.uniform(-0.5, 1.5, n)])
        if n > 10:
            p[::7, 0] = np.round(p[::7, 0], 3)          # exact-mm values (truncation boundary)
        frames.append({"frame_id": 3 * i + 1, "timestamp": 0.05 * i + 1e-3, "points": p})
    assert mc.codecs.encode_lvx(frames, gpu_ctx) == C.lvx_bytes(frames)


@pytest.mark.parametrize("case", ["tricky", "specials", "random", "f32", "empty", "wide"])
def test_pcd_matches_reference_bytes(mc, gpu_ctx, tmp_path, case):
    g = golden("codecs.npz")
    pts = g[f"pcd/{case}/points"]
    want = g[f"pcd/{case}/bytes"].tobytes()
    fn = str(tmp_path / f"{case}.pcd")
    mc.codecs.save_pcd(pts, fn, gpu_ctx)
    with open(fn, "rb") as f:
        assert f.read() == want


def test_pcd_batched_frames_long_lines_and_limits(mc, gpu_ctx):
    g = golden("codecs.npz")
    rng = np.random.default_rng(8)
    mags = 10.0 ** rng.uniform(-12, 31, (3000, 4))
    huge = rng.choice([-1, 1], (3000, 4)) * mags           # lines up to ~150 B: exceeds the LDS tile
    ties = (rng.integers(-2 ** 20, 2 ** 20, (1000, 4)) / 128.0)   # many exact half-way cases
    clouds = [g["pcd/tricky/points"], huge, np.zeros((0, 4)), ties, g["pcd/random/points"]]
    got = mc.codecs.encode_pcd_frames(clouds, gpu_ctx)
    for c, b in zip(clouds, got):
        assert b == C.pcd_ascii_bytes(c)
    with pytest.raises(ValueError):
        mc.codecs.encode_pcd(np.array([[1e33, 0, 0, 0]]), gpu_ctx)
    with pytest.raises(IndexError):
        mc.codecs.encode_pcd(np.zeros((2, 3)), gpu_ctx)


def test_pcd_packed_path_digit_boundaries_and_mixed_tiles(mc, gpu_ctx):
    """The packed line path (|v| < 4294, not within 1e-6 of a %.6f tie) against the oracle: every
    integer-digit count and sign, values that round across a digit boundary, -0.0, near-ties on
    either side of the 1e-6 guard, and 256-line tiles holding one byte-path line (first, middle,
    last line of the tile) beside packed-only tiles."""
    rng = np.random.default_rng(21)
    edges = np.array([0.0, -0.0, 1e-7, 4.9e-7, 5e-7, 5.1e-7, 9.9999994, 9.9999995, 9.9999996, 99.9999996,
                      999.9999996, 999.9999994, 1000.0, 4293.999999, 4293.9999996, 4294.0, 4294.5,
                      0.1234565, 0.12345650001, 1.0000005, 1.00000049, 12.3456785])
    edges = np.concatenate([edges, -edges])
    mags = 10.0 ** rng.uniform(-8, np.log10(4293.9), (40_000, 4))
    vals = rng.choice([-1.0, 1.0], mags.shape) * mags
    vals[:len(edges), 0] = edges
    vals[:len(edges), 1] = edges[::-1]
    vals[:, 3] = np.where(np.arange(len(vals)) % 3 == 0, rng.uniform(0, 1, len(vals)), vals[:, 3])
    for pos in (0, 1000, 1279, 256 * 10 + 128, 256 * 20 + 255, 39_999):
        vals[pos, pos % 4] = 1e7 * (1 + pos)                  # one byte-path line in this tile
    clouds = [vals[:1], vals[1:256], vals[256:512], vals[512:769], vals[769:], vals[:300] * 0.001]
    got = mc.codecs.encode_pcd_frames(clouds, gpu_ctx)
    for c, b in zip(clouds, got):
        assert b == C.pcd_ascii_bytes(c)


def test_codecs_from_device_batch(mc, gpu_ctx):
    counts = np.array([1000, 0, 2500, 96], np.int64)
    b = gpu_ctx.batch(counts, with_time=True)
    b.synth(seed=3, frame_id_base=50)
    host = b.split(b.download_aos())
    pcds = mc.codecs.encode_pcd_batch(b)
    for h, p in zip(host, pcds):
        assert p == C.pcd_ascii_bytes(h)
    ids, ts = [5, 6, 7, 8], [0.1, 0.2, 0.3, 0.4]
    lvx = mc.codecs.encode_lvx_batch(b, ids, ts)
    ref = C.lvx_bytes([{"frame_id": i, "timestamp": t, "points": h} for i, t, h in zip(ids, ts, host)])
    assert lvx == ref


@pytest.mark.parametrize("with_time", [False, True])
def test_batch_source_encoders_match_f64_source(mc, gpu_ctx, with_time):
    """mc_*_encode_batch read the batch's blocked float32 columns (4 or 5 per block); their bytes
    must equal the f64-AoS encoders' on the same values: ragged frames across block boundaries,
    half-way ties, inf, large magnitudes."""
    rng = np.random.default_rng(8)
    counts = np.array([255, 256, 257, 0, 1, 70_001], np.int64)
    n = int(counts.sum())
    pts = rng.normal(0, 50, (n, 4))
    pts[:300] = rng.integers(-2 ** 20, 2 ** 20, (300, 4)) / 128.0          # exact f32 ties at 1e-6
    pts[300:310] = np.array([np.inf, -np.inf, 1e30, -3.4e30])[rng.integers(0, 4, (10, 4))]
    fin = np.isfinite(pts[:, 3])
    pts[fin, 3] = np.abs(pts[fin, 3]) % 1.0                                 # inf stays inf
    b = gpu_ctx.batch(counts, with_time=with_time)
    b.upload_aos(pts)
    host = b.split(b.download_aos())
    assert [len(h) for h in host] == list(counts)
    assert mc.codecs.encode_pcd_batch(b) == mc.codecs.encode_pcd_frames(host, gpu_ctx)
    assert mc.codecs.encode_pcd_batch(b)[1] == C.pcd_ascii_bytes(host[1])
    ok = np.isfinite(pts).all(axis=1) & (np.abs(pts) < 2e6).all(axis=1)
    b2 = gpu_ctx.batch(counts, with_time=with_time)
    b2.upload_aos(np.where(ok[:, None], pts, 1.5))
    h2 = b2.split(b2.download_aos())
    ids, ts = np.arange(6) + 40, np.arange(6) * 0.05
    lvx = mc.codecs.encode_lvx_batch(b2, ids, ts)
    assert lvx == mc.codecs.encode_lvx([{"frame_id": i, "timestamp": t, "points": h}
                                        for i, t, h in zip(ids, ts, h2)], gpu_ctx)
    # clipping (LMC:259-261, 268): coordinates past +-2^31 mm, intensities outside [0, 1]; frames of
    # 1 / 767 / 768 / 769 / 1537 points (a k_lvx_packages unit is 768 points = 3 blocks; a frame's
    # first unit writes its frame header)
    cc = np.array([767, 1, 768, 769, 1537], np.int64)
    m = int(cc.sum())
    clip = np.column_stack([rng.normal(0, 40, (m, 3)), rng.uniform(-0.3, 1.3, m)])
    clip[::7, 0] = 3e6
    clip[::11, 1] = -3e6
    clip[::13, 2] = 2147483.5
    b3 = gpu_ctx.batch(cc, with_time=with_time)
    b3.upload_aos(clip)
    h3 = b3.split(b3.download_aos())
    ids3, ts3 = np.arange(5) + 7, np.arange(5) * 0.1 + 3.0
    assert mc.codecs.encode_lvx_batch(b3, ids3, ts3) == mc.codecs.encode_lvx(
        [{"frame_id": i, "timestamp": t, "points": h} for i, t, h in zip(ids3, ts3, h3)], gpu_ctx)
    nan = gpu_ctx.batch([3])
    nan.upload_aos(np.array([[1.0, np.nan, 0, 0.5], [0, 0, 0, 0], [1, 1, 1, 1]]))
    with pytest.raises(ValueError):                 # the reference's int(nan) (LMC:259)
        mc.codecs.encode_lvx_batch(nan, [0], [0.0])
    nan2 = gpu_ctx.batch([800])                     # a NaN intensity in the second unit
    v = np.column_stack([rng.normal(0, 10, (800, 3)), rng.uniform(0, 1, 800)])
    v[790, 3] = np.nan
    nan2.upload_aos(v)
    with pytest.raises(ValueError):
        mc.codecs.encode_lvx_batch(nan2, [0], [0.0])


def test_simulator_save_lvx_and_pcd(mc, gpu_ctx, tmp_path):
    sim = mc.LiDARMotionSimulator(context=gpu_ctx)
    rng = np.random.default_rng(1)
    scans = [{"frame_id": i, "timestamp": 0.1 * i, "points_local": rng.normal(0, 20, (n, 4))}
             for i, n in enumerate([10, 0, 200])]
    base = str(tmp_path / "run")
    sim.save_lvx({"raw_scans": scans}, base)
    with open(base + ".lvx", "rb") as f:
        data = f.read()
    assert data == C.lvx_bytes([{"frame_id": s["frame_id"], "timestamp": s["timestamp"],
                                 "points": s["points_local"]} for s in scans])
    sim.save_pcd(scans[2]["points_local"], os.path.join(tmp_path, "f.pcd"))
    with open(os.path.join(tmp_path, "f.pcd"), "rb") as f:
        assert f.read() == C.pcd_ascii_bytes(scans[2]["points_local"])


@pytest.mark.parametrize("tag", ["gap", "full"])
def test_save_results_files_match_reference(mc, gpu_ctx, tmp_path, tag):
    """LMC:860-931: every file save_results writes (CSVs, per-frame and merged PCDs, LVX), byte for
    byte against the reference's own output directory (tests/golden/save_results.npz)."""
    g = golden("save_results.npz")
    cols = [str(c) for c in g["in/motion_cols"]]
    motion = []
    for row in g["in/motion"]:
        m = {c: float(v) for c, v in zip(cols, row)}
        m["frame_id"] = int(m["frame_id"])
        motion.append(m)
    raw = []
    i = 0
    while f"{tag}/in/raw/{i}" in g:
        fid = int(g[f"{tag}/in/frame_id/{i}"])
        raw.append({"frame_id": fid, "timestamp": 0.1 * fid, "points_local": g[f"{tag}/in/raw/{i}"]})
        i += 1
    aligned = []
    i = 0
    while f"{tag}/in/aligned/{i}" in g:
        aligned.append(g[f"{tag}/in/aligned/{i}"])
        i += 1
    tr = {k: g[f"in/trajectory/{k}"] for k in ("time", "position", "position_gps")}
    results = {"raw_scans": raw, "aligned_pointclouds": aligned, "motion_data": motion, "trajectory": tr}
    sim = mc.LiDARMotionSimulator(context=gpu_ctx)
    sim.save_results(results, str(tmp_path))
    want = {k[len(tag) + 1:]: g[k].tobytes() for k in g.files if k.startswith(tag + "/") and "/in/" not in k}
    got = {}
    for root, _, files in os.walk(tmp_path):
        for fn in files:
            p = os.path.join(root, fn)
            with open(p, "rb") as f:
                got[os.path.relpath(p, tmp_path)] = f.read()
    assert sorted(got) == sorted(want)
    for k in want:
        assert got[k] == want[k], k


def _deskew_setup(mc, ctx, counts, with_big=False):
    sim = mc.LiDARMotionSimulator({"duration": 20.0, "trajectory_type": "figure_eight", "max_speed": 12.0},
                                  context=ctx)
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:len(counts)]
    b = ctx.batch(counts, with_time=True)
    b.synth(seed=4, frame_id_base=700)
    if with_big:   # a frame with values beyond the packed formatter (|v| >= 4294 after the deskew)
        pts = b.download_aos()
        t_ns = b.download_time()
        pts[:50, 0] = 6000.0
        b.upload_aos(pts)
        b.upload_time(t_ns)
    b.set_frame_times(times)
    b.set_frame_starts((times * 1e9).astype(np.int64))
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    ts, gyro = mc.trajectory.imu_from_trajectory(tr, 200.0)
    ctx.set_imu(ts, gyro)
    return b


@pytest.mark.parametrize("mode", ["frame", "pose_slerp", "imu"])
@pytest.mark.parametrize("big", [False, True])
def test_deskew_pcd_equals_deskew_then_encode(mc, gpu_ctx, mode, big):
    """mc_deskew_pcd (the deskew kernel sums each block's PCD text bytes, the writer skips its
    measure pass) produces the same deskewed batch and the same PCD bytes as mc_deskew followed by
    mc_pcd_encode_batch: ragged frames (empty, < 4, one block, a block + 1, several tiles); with
    ``big`` a frame holds values >= 4294, whose blocks take the measure-pass fallback."""
    counts = np.array([4096, 3, 2500, 0, 10_000, 7, 256, 257, 100_003, 1], np.int64)
    b = _deskew_setup(mc, gpu_ctx, counts, with_big=big)
    ref_out = gpu_ctx.deskew(b, gpu_ctx.batch(counts), mode=mode)
    want = mc.codecs.encode_pcd_batch(ref_out)
    out = gpu_ctx.batch(counts)
    gpu_ctx.sync()
    gpu_ctx.read_timing()
    gpu_ctx.timing(True)
    got = mc.codecs.deskew_pcd_frames(b, out, mode=mode)
    gpu_ctx.timing(False)
    tm = gpu_ctx.read_timing()
    assert np.array_equal(out.download_aos(), ref_out.download_aos())
    assert len(got) == len(want)
    for f, (g, w) in enumerate(zip(got, want)):
        assert g == w, (mode, f)
    # fast case: the write pass only (one codec launch); fallback: measure + write (+ the byte path)
    assert tm["codec_launches"] >= 2 if big else tm["codec_launches"] == 1
    assert tm["main_launches"] == 1


def test_deskew_pcd_space_and_errors(mc, gpu_ctx):
    counts = np.array([300, 0, 1000], np.int64)
    b = _deskew_setup(mc, gpu_ctx, counts)
    out = gpu_ctx.batch(counts)
    small = gpu_ctx.device_buffer(64)
    text, pos = mc.codecs.deskew_pcd_batch(b, out, mode="frame", text=small)   # regrows after MC_ERR_SPACE
    body = text.to_host(np.uint8, count=int(pos[-1])).tobytes()
    text.close()
    want = mc.codecs.encode_pcd_batch(gpu_ctx.deskew(b, gpu_ctx.batch(counts), mode="frame"))
    assert [mc.codecs.pcd_header(int(c)) + body[pos[f]:pos[f + 1]] for f, c in enumerate(counts)] == want
    with pytest.raises(ValueError):
        mc.codecs.deskew_pcd_batch(b, b, mode="frame")
    with pytest.raises(ValueError):
        mc.codecs.deskew_pcd_batch(b, gpu_ctx.batch([300, 1, 1000]), mode="frame")


def test_pcd_batch_many_tiles_space_and_sizes(mc, gpu_ctx):
    """mc_pcd_encode_batch over thousands of tiles (several tiles per write workgroup, the next
    tile's values converted before the current tile's stores), empty frames between full ones, a
    tile holding byte-path lines among packed ones, against the f64-AoS encoder and the oracle; a
    buffer one byte short returns MC_ERR_SPACE with the exact size, a NULL buffer only the sizes."""
    from ctypes import c_int64
    rng = np.random.default_rng(77)
    counts = np.array([1000] * 150 + [0, 0] + [300, 1, 0, 4096] * 20 + [777], np.int64)
    n = int(counts.sum())
    pts = np.column_stack([rng.normal(0, 300, (n, 3)), rng.uniform(0, 1, n)])
    pts[50_000:50_003, 1] = [5000.0, -1e9, np.inf]                      # one partition takes the byte path
    b = gpu_ctx.batch(counts)
    b.upload_aos(pts)
    host = b.split(b.download_aos())
    got = mc.codecs.encode_pcd_batch(b)
    assert got == mc.codecs.encode_pcd_frames(host, gpu_ctx)
    for f in (0, 49, 50, 150, 151, 152, 153, len(counts) - 1):
        assert got[f] == C.pcd_ascii_bytes(host[f])
    lib, ptr = gpu_ctx.lib, mc._lib.ptr
    pos = np.zeros(len(counts) + 1, np.int64)
    assert lib.mc_pcd_encode_batch(gpu_ctx.handle, b.handle, None, 0, ptr(pos, c_int64)) == mc._lib.MC_ERR_SPACE
    total = int(pos[-1])
    assert total == sum(len(g) - len(mc.codecs.pcd_header(int(c))) for g, c in zip(got, counts))
    buf = gpu_ctx.device_buffer(total)
    try:
        assert lib.mc_pcd_encode_batch(gpu_ctx.handle, b.handle, buf.ptr, total - 1, ptr(pos, c_int64)) == \
            mc._lib.MC_ERR_SPACE
        assert int(pos[-1]) == total
        assert lib.mc_pcd_encode_batch(gpu_ctx.handle, b.handle, buf.ptr, total, ptr(pos, c_int64)) == 0
        text = buf.to_host(np.uint8, count=total).tobytes()
    finally:
        buf.close()
    for f, c in enumerate(counts):
        assert mc.codecs.pcd_header(int(c)) + text[pos[f]:pos[f + 1]] == got[f]


@pytest.mark.parametrize("mode", ["pose_slerp", "frame"])
def test_codec_unit_orders_give_the_same_bytes(mc, gpu_ctx, mode):
    """The codec launches start where the last kernel over the batch ended (mc_batch::hot_order,
    layout.hpp stream_unit): after a deskew in dealt order (SLERP) or in XCD ranges (frame mode),
    encodes in a row run the batch forwards and backwards, whole or by XCD range; every file must
    equal the oracle's (ragged frames, an empty one, partial units and tiles)."""
    counts = np.array([4096, 3, 2500, 0, 10_000, 7, 256, 257, 20_003, 1], np.int64)
    b = _deskew_setup(mc, gpu_ctx, counts)
    out = gpu_ctx.deskew(b, gpu_ctx.batch(counts), mode=mode)
    host = out.split(out.download_aos())
    want_pcd = [C.pcd_ascii_bytes(h) for h in host]
    ids, ts = np.arange(len(counts)) + 90, np.arange(len(counts)) * 0.1
    want_lvx = C.lvx_bytes([{"frame_id": i, "timestamp": t, "points": h} for i, t, h in zip(ids, ts, host)])
    for _ in range(2):   # each call flips the direction of the next
        assert mc.codecs.encode_pcd_batch(out) == want_pcd
        assert mc.codecs.encode_lvx_batch(out, ids, ts) == want_lvx
    assert mc.codecs.deskew_pcd_frames(b, out, mode=mode) == want_pcd


def _encode_timed(mc, ctx, b):
    ctx.sync()
    ctx.read_timing()
    ctx.timing(True)
    got = mc.codecs.encode_pcd_batch(b)
    ctx.timing(False)
    return got, ctx.read_timing()["codec_launches"]


@pytest.mark.parametrize("mode", ["frame", "pose_slerp", "imu"])
@pytest.mark.parametrize("big", [False, True])
def test_pcd_len_batch_deskew_then_encode(mc, gpu_ctx, mode, big):
    """MC_BATCH_WITH_PCD_LEN: a deskew into the batch (mc_deskew and the last launch of
    mc_deskew_steps) leaves its blocks' text sums, so mc_pcd_encode_batch runs the write pass only
    and writes the bytes a plain batch gets through measure + write; a block with a value beyond the
    packed formatter falls back to the measure pass."""
    counts = np.array([4096, 3, 2500, 0, 10_000, 7, 256, 257, 100_003, 1], np.int64)
    b = _deskew_setup(mc, gpu_ctx, counts, with_big=big)
    plain = gpu_ctx.deskew(b, gpu_ctx.batch(counts), mode=mode)
    want = mc.codecs.encode_pcd_batch(plain)
    out = gpu_ctx.batch(counts, with_pcd_len=True)
    assert not out.pcd_len_current()
    for issue in ("deskew", "steps"):
        if issue == "deskew":
            gpu_ctx.deskew(b, out, mode=mode)
        else:
            gpu_ctx.deskew_steps(b, out, 3, mode=mode)
        assert out.pcd_len_current()
        got, launches = _encode_timed(mc, gpu_ctx, out)
        assert got == want, (mode, issue)
        assert launches >= 2 if big else launches == 1, (mode, issue, launches)
    assert np.array_equal(out.download_aos(), plain.download_aos())
    # mc_deskew_pcd into the same kind of batch: the batch's own sums, then the write pass
    assert mc.codecs.deskew_pcd_frames(b, out, mode=mode) == want
    assert out.pcd_len_current()
    # any other write of the columns makes the sums stale: the encoder measures again
    gpu_ctx.tune_order(b, out, mode=mode, launches=2, rounds=2)
    assert not out.pcd_len_current()
    got, launches = _encode_timed(mc, gpu_ctx, out)
    assert got == want and launches >= 2


@pytest.mark.parametrize("ld", [4, 6])
def test_pcd_len_batch_stager_and_stale_writes(mc, gpu_ctx, ld):
    """The stager (AoS float64 -> columns, ld 4 and wider rows) writes the sums too; column uploads,
    synth and affine writes leave them stale.  Bytes always equal the oracle's."""
    rng = np.random.default_rng(12)
    counts = np.array([255, 256, 257, 0, 1, 5000, 2049], np.int64)
    n = int(counts.sum())
    pts = np.column_stack([rng.normal(0, 80, (n, 3)), rng.uniform(0, 1, n), rng.normal(0, 1, (n, ld - 4))])
    pts[7, 0] = -0.0
    pts[300, 1] = 999.9999996      # rounds up to 1000.000000 at six decimals (f32: 1000.0)
    b = gpu_ctx.batch(counts, with_pcd_len=True)
    b.upload_aos(pts)
    assert b.pcd_len_current()
    host = b.split(b.download_aos())
    got, launches = _encode_timed(mc, gpu_ctx, b)
    assert launches == 1
    assert got == [C.pcd_ascii_bytes(h) for h in host]
    x, y, z, i = b.download_columns()
    b.upload_columns(x=x * 2)
    assert not b.pcd_len_current()
    host2 = b.split(b.download_aos())
    got, launches = _encode_timed(mc, gpu_ctx, b)
    assert launches >= 2 and got == [C.pcd_ascii_bytes(h) for h in host2]
    b.upload_aos(pts)
    assert b.pcd_len_current()
    b.synth(seed=1)
    assert not b.pcd_len_current()
    b.upload_aos(pts)
    gpu_ctx.transform_affine(b, b, np.eye(4)[:3])
    assert not b.pcd_len_current()
    # a slow value through the stager: sums current, but the encoder must still measure that block
    pts[5100, 2] = 1e7
    b.upload_aos(pts)
    host3 = b.split(b.download_aos())
    got, launches = _encode_timed(mc, gpu_ctx, b)
    assert launches >= 2 and got == [C.pcd_ascii_bytes(h) for h in host3]


def test_pcd_len_batch_scan_emit(mc, gpu_ctx):
    """mc_scan_emit into a MC_BATCH_WITH_PCD_LEN batch adds each point's text bytes to its block
    (atomics into zeroed slots): write pass only, bytes as the oracle's."""
    sim = mc.LiDARMotionSimulator({"points_per_frame": 3000, "lidar_range_noise": 0.01}, context=gpu_ctx)
    rng = np.random.default_rng(3)
    env = np.column_stack([rng.uniform(-80, 80, (60_000, 3)), rng.uniform(0, 1, 60_000)])
    env[:, 2] *= 0.1
    sim._load_environment(env)
    times = np.linspace(0, 10, 9)
    tr = {"time": times, "position_gps": rng.normal(0, 3, (9, 3)), "orientation_imu": rng.normal(0, 0.3, (9, 3))}
    gpu_ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    np.random.seed(5)
    counts, noise = gpu_ctx._scan_count(times, sim.config, "searchsorted", np.random)
    out = gpu_ctx.batch(counts, with_pcd_len=True)
    mc._lib.check(gpu_ctx.lib.mc_scan_emit(gpu_ctx.handle, out.handle, mc._lib.ptr(noise, mc._lib.c_double)), "emit")
    assert out.pcd_len_current()
    host = out.split(out.download_aos())
    got, launches = _encode_timed(mc, gpu_ctx, out)
    assert launches == 1
    assert got == [C.pcd_ascii_bytes(h) for h in host]


@pytest.mark.parametrize("ld", [4, 6])
def test_pcd_len_sums_at_the_length_boundaries(mc, gpu_ctx, ld):
    """The summing stager's text lengths (layout.hpp PcdCount) on the float32 neighbours of every
    value where "%.6f" changes length (tests/test_pcd_len_rule.py checks the rule itself on the CPU),
    ±0, denormals and both signs: write pass only, bytes equal to the oracle's; the same values past
    the slow mark (4288) send their blocks to the measure pass and still match."""
    def around(b, k=48):
        c = np.float32(b).view(np.int32)
        v = np.arange(c - k, c + k + 1, dtype=np.int32).view(np.float32)
        return np.concatenate([v, -v])
    vals = np.concatenate([around(b) for b in (5e-7, 1e-6, 1.0, 10.0, 100.0, 1000.0, 4287.0)]
                          + [np.array([0.0, -0.0, 1e-45, -1e-45, 1.1754942e-38, -1.1754942e-38], np.float32)])
    rng = np.random.default_rng(21)
    for extra, launches_ok in ((np.zeros(0, np.float32), lambda k: k == 1),
                               (np.array([4288.0, -4293.9, 1e6, np.inf], np.float32), lambda k: k >= 2)):
        v = np.concatenate([vals, extra]).astype(np.float64)
        n = -(-v.size // 4)
        cols = np.resize(rng.permutation(v), 4 * n).reshape(n, 4)     # every value in some column
        pts = np.column_stack([cols, rng.normal(0, 1, (n, ld - 4))]) if ld > 4 else cols
        counts = np.array([n // 3, 0, n - n // 3 - 5, 5], np.int64)
        b = gpu_ctx.batch(counts, with_pcd_len=True)
        b.upload_aos(pts)
        assert b.pcd_len_current()
        host = b.split(b.download_aos())
        got, launches = _encode_timed(mc, gpu_ctx, b)
        assert launches_ok(launches), launches
        assert got == [C.pcd_ascii_bytes(h) for h in host]
