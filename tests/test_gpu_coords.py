"""GPU CoordinateTransformer (CSIM:153-233) and _transform_coordinates (CSIM:2107-2163) against the
reference's own outputs (tests/golden/coords.npz).  The points stay float64 end to end
(mc_affine_rows_f64, numpy's accumulation order): with the reference's matrix the outputs equal
the reference's bit for bit; with matrices this box's numpy builds (CoordinateTransformer's
Rz @ Ry @ Rx, np.linalg.inv), they are held to the strict per-coordinate 1e-5 (and are bitwise
equal wherever those matrices are)."""
import numpy as np
import pytest

from conftest import assert_scaled_close, golden, scale_of
from oracle import restatement as R

pytestmark = pytest.mark.gpu


def check(out, want, p, T, what):
    """strict per-coordinate parity; bitwise when this box built the reference's very matrix"""
    assert out.dtype == np.float64 and out.shape == want.shape, what
    assert_scaled_close(out, want, scale_of(np.asarray(p)[:, :3], T[:3, 3]), what=what)
    return bool(np.array_equal(out, want))


def test_transform_points_matches_reference(mc, gpu_ctx):
    g = golden("coords.npz")
    ct = mc.CoordinateTransformer(gpu_ctx)
    ct.set_transformation("sensor", "local", [10.0, -5.0, 2.0], [0.1, -0.2, 2.5])
    np.testing.assert_allclose(ct.transformations[("sensor", "local")], g["T/sensor/local"], atol=1e-15)
    p3 = g["p3"]
    for a, b in [("sensor", "vehicle"), ("sensor", "local"), ("local", "sensor"), ("sensor", "sensor")]:
        T = ct.transformations[(a, b)]
        out = ct.transform_points(p3, a, b)
        assert out.shape == (200, 3)
        same = check(out, g[f"tp/{a}/{b}"], p3, T, f"{a}->{b}")
        ref_T = {("sensor", "local"): "T/sensor/local", ("local", "sensor"): "T/local/sensor"}.get((a, b))
        if ref_T is None or np.array_equal(T, g[ref_T]):
            assert same, f"{a}->{b}: the reference's matrix but not its bits"
        assert_scaled_close(out, R.transform_points_h(p3, T), scale_of(p3, T[:3, 3]), what=f"{a}->{b} oracle")
    # homogeneous (N,4): the 4th column is w
    out4 = ct.transform_points(g["p4"], "sensor", "local")
    T = ct.transformations[("sensor", "local")]
    same = check(out4, g["tp4/sensor/local"], g["p4"], T, "homogeneous")
    assert same or not np.array_equal(T, g["T/sensor/local"])
    # (1, 3) calls: numpy's matrix-vector order, as _transform_coordinates' per-point loop recorded it
    xyz = g["tc/in/0"]
    one = np.vstack([ct.transform_points(xyz[j:j + 1], "sensor", "local") for j in range(len(xyz))])
    if np.array_equal(ct.transformations[("sensor", "local")], g["T/sensor/local"]):
        assert np.array_equal(one, g["tc/local/0"]), int(np.count_nonzero(one != g["tc/local/0"]))
    # missing pair: a warning and the very same array back
    assert ct.transform_points(p3, "vehicle", "sensor") is p3
    with pytest.raises(ValueError):
        ct.transform_points(np.zeros((4, 5)), "sensor", "local")
    assert ct.transform_points(np.zeros((0, 3)), "sensor", "vehicle").shape == (0, 3)


def test_reference_matrices_give_reference_bits(mc, gpu_ctx):
    """The device arithmetic alone: the reference's own 4x4 matrices (as recorded) applied by
    transform_arrays reproduce its outputs exactly — including a UTM-scale translation (easting /
    northing 5.1e5 / 4.4e6 m), where float32 points would be quantised to 0.5 m."""
    g = golden("coords.npz")
    cases = [(g["p3"], g["T/sensor/local"], g["tp/sensor/local"]),
             (g["p3"], g["T/local/sensor"], g["tp/local/sensor"]),
             (g["p4"], g["T/sensor/local"], g["tp4/sensor/local"]),
             (g["big/p3"], g["big/T"], g["big/fwd"]),
             (g["big/fwd"], g["big/T_inv"], g["big/back"])]
    for i, (p, T, want) in enumerate(cases):
        out = mc.coords.transform_arrays([p], T, context=gpu_ctx)[0]
        assert np.array_equal(out, want), (i, int(np.count_nonzero(out != want)), float(np.abs(out - want).max()))
    # the big round trip returns within float64 noise of the input (not 0.5 m)
    assert np.abs(g["big/back"] - g["big/p3"]).max() < 1e-8


def test_utm_scale_translation_strict_vs_oracle(mc, gpu_ctx):
    """CoordinateTransformer with translation (5e5, 4.43e6, 0) built on this box: strict per
    coordinate against the oracle."""
    ct = mc.CoordinateTransformer(gpu_ctx)
    ct.set_transformation("sensor", "utm", [5e5, 4.43e6, 0.0], [0.02, -0.01, 2.2])
    rng = np.random.default_rng(8)
    p = rng.normal(0, 60, (50_000, 3))
    for a, b in (("sensor", "utm"), ("utm", "sensor")):
        T = ct.transformations[(a, b)]
        src = p if a == "sensor" else R.transform_points_h(p, ct.transformations[("sensor", "utm")])
        out = ct.transform_points(src, a, b)
        assert_scaled_close(out, R.transform_points_h(src, T), scale_of(src, T[:3, 3]), what=f"{a}->{b}")
    back = ct.transform_points(ct.transform_points(p, "sensor", "utm"), "utm", "sensor")
    assert np.abs(back - p).max() < 1e-8


def test_transform_coordinates_matches_reference(mc, gpu_ctx):
    g = golden("coords.npz")
    ct = mc.CoordinateTransformer(gpu_ctx)
    ct.set_transformation("sensor", "local", [10.0, -5.0, 2.0], [0.1, -0.2, 2.5])
    frames = []
    for i in range(int(g["tc/n_frames"])):
        xyz = g[f"tc/in/{i}"]
        pts = [mc.LiDARPoint(x=float(x), y=float(y), z=float(z), intensity=k % 256, timestamp=1_000_000 * k,
                             ring=0, tag=0) for k, (x, y, z) in enumerate(xyz)]
        frames.append({"frame_id": i, "timestamp": i * 100_000_000, "points": pts})
    gps = [mc.GPSData(0, 40.0, -74.0, 10.0, 0.0, 0.0, 0.0, 0.0)]
    for target in ("vehicle", "local", "utm"):
        res = mc.coords.transform_coordinates(frames, target, gps, ct)
        for i, fr in enumerate(res):
            got = np.array([[p.x, p.y, p.z] for p in fr["points"]]).reshape(-1, 3)
            want = g[f"tc/{target}/{i}"]
            T = ct.transformations.get(("sensor", target), np.eye(4))
            same = check(got, want, g[f"tc/in/{i}"], T, f"{target}/{i}")
            if target != "local" or np.array_equal(T, g["T/sensor/local"]):
                assert same, f"{target}/{i}"
            meta = np.array([[p.intensity, p.timestamp] for p in fr["points"]], np.int64).reshape(-1, 2)
            assert np.array_equal(meta, g[f"tc/{target}/{i}/meta"])
            assert fr["coordinate_system"] == target and fr["frame_id"] == i


def test_transform_arrays_per_frame_matrices_large(mc, gpu_ctx):
    rng = np.random.default_rng(4)
    counts = [0, 5, 100_003, 77, 250_000]
    frames = [rng.normal(0, 50, (n, 3)) for n in counts]
    Ts = np.stack([R.create_transform_matrix(rng.normal(0, 100, 3), rng.uniform(-np.pi, np.pi, 3)) for _ in counts])
    out = mc.coords.transform_arrays(frames, Ts, context=gpu_ctx)
    for f, T, o in zip(frames, Ts, out):
        assert o.shape == (len(f), 3)
        assert_scaled_close(o, R.transform_points_h(f, T), scale_of(f, T[:3, 3]))
    # homogeneous rows, one matrix per frame, above the zero-copy size
    h = [np.column_stack([f, rng.uniform(0.5, 2, len(f))]) for f in frames]
    out = mc.coords.transform_arrays(h, Ts, context=gpu_ctx)
    for f, T, o in zip(h, Ts, out):
        assert_scaled_close(o, R.transform_points_h(f, T), scale_of(f[:, :3], T[:3, 3]) * 2)


def test_utm_offset_is_a_plain_add(mc, gpu_ctx, monkeypatch):
    """CSIM:2132 `point_array[0] + np.array([utm_x, utm_y, 0])`: each coordinate one add, so a NaN or
    inf in one coordinate stays there and -0.0 + 0 gives 0.0 — bit for bit with numpy on the device
    (MC_AFFINE_TRANSLATE), directly and through transform_coordinates' UTM branch (a stand-in `utm`
    module: the package is not installed here, and without it the reference leaves points unchanged)."""
    rng = np.random.default_rng(6)
    p = rng.normal(0, 40, (1000, 3))
    p[3] = [np.nan, 1.0, 2.0]
    p[4] = [1.0, np.inf, -3.0]
    p[5] = [-0.0, -0.0, -0.0]
    off = np.array([583_960.123456789, 4_507_523.98765, 0.0])
    got = gpu_ctx.affine_rows([len(p)], p, np.column_stack([np.eye(3), off]), translate=True)
    want = p + np.array([off[0], off[1], 0])
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))

    class FakeUtm:
        @staticmethod
        def from_latlon(lat, lon):
            return 583_960.0 + lat, 4_507_523.0 + lon, 18, "T"
    monkeypatch.setattr(mc.coords, "UTM_AVAILABLE", True)
    monkeypatch.setattr(mc.coords, "utm", FakeUtm, raising=False)
    ct = mc.CoordinateTransformer(gpu_ctx)
    frames = []
    for i in range(3):
        xyz = p[i * 300:(i + 1) * 300 + (5 if i == 0 else 0)]
        pts = [mc.LiDARPoint(x=float(x), y=float(y), z=float(z), intensity=1, timestamp=k, ring=0, tag=0)
               for k, (x, y, z) in enumerate(xyz)]
        frames.append({"frame_id": i, "timestamp": i * 100_000_000, "points": pts})
    gps = [mc.GPSData(0, 40.5, -74.25, 10.0, 0.0, 0.0, 0.0, 0.0),
           mc.GPSData(150_000_000, 40.75, -74.5, 10.0, 0.0, 0.0, 0.0, 0.0)]
    res = mc.coords.transform_coordinates(frames, "utm", gps, ct)
    for fr, src in zip(res, frames):
        s = mc.coords.find_closest_gps_sample(gps, src["timestamp"])
        ux, uy, _, _ = FakeUtm.from_latlon(s.latitude, s.longitude)
        xyz = np.array([[q.x, q.y, q.z] for q in src["points"]])
        want = xyz + np.array([ux, uy, 0])
        got = np.array([[q.x, q.y, q.z] for q in fr["points"]])
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
