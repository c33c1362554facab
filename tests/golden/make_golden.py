"""Generate the golden vectors in tests/golden/ by running the reference itself.

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference (/root/reference, read-only) is imported with a stub ``laspy`` module: LMC:12
imports laspy unconditionally but uses it only in ``save_las`` (LMC:950-963), off the path.
Only inputs and outputs are written (npz / json data); no reference source is copied.

Fixtures:
  lmc_frames.npz      Path A: selected frames of the three LMC scenarios — local scan, selected
                      pose index / position / rpy, frame time, reference aligned output.
  lmc_traj_<cfg>.npz  trajectory tables (LMC:361-428) with the reference's seed-42 noise.
  lmc_kat.npz         transform_pointcloud known-answer cases (zero rotation, yaw=pi/2, ...).
  lmc_config.json     LiDARMotionSimulator config defaults and validation errors (LMC:297-359).
  csim_pathb.npz      Path B: CSIM IMU stream + points + compensate_point_cloud output, with the
                      before-first / after-last / duplicate-timestamp edge cases.
  slerp.npz           build-added SLERP mode: scipy Slerp + LERP over a parking interval that
                      straddles the yaw wrap (not a reference function: anchored on scipy).
  synth.npz           first 4096 points and f64 column sums of a synthetic 100k frame.
  lmc_env_<cfg>.npz   scan_environment (LMC:701-770): the scenario's scene and numpy's RNG state
                      right before the frame loop, plus every frame's point count.
  codecs.npz          LVX v1.1 files (write_compatible_lvx, LMC:57-272) and ASCII PCD files
                      (save_pcd, LMC:932-948) written by the reference, with their inputs.
  coords.npz          CoordinateTransformer matrices / transforms and _transform_coordinates
                      (CSIM:153-233, 2107-2163).
  save_results.npz    the whole output directory of LMC's save_results (LMC:860-931).
  lmc_run_files.json  the reference's own end-to-end runs: for each scenario, run_simulation()
                      (LMC:778-858) then save_results() (LMC:860-931); every file of the output
                      directory by relative path -> [size, sha256], the printed log, and per-frame
                      point counts.  The scene and the RNG state before the frame loop are
                      lmc_env_<cfg>.npz (checked here to be the same run).
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.path.insert(0, REPO)


def import_reference():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("laspy", types.ModuleType("laspy"))
    sys.path.insert(0, REF)
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        import lidar_motion_compensation as lmc  # noqa: E402
        import livox_mid70_complete_simulator as csim  # noqa: E402
    return lmc, csim


SCENARIOS = {  # LMC:1182-1204
    "urban_complex": {"duration": 120.0, "trajectory_type": "figure_eight",
                      "environment_complexity": "complex", "max_speed": 12.0, "lidar_fps": 10},
    "highway_simple": {"duration": 60.0, "trajectory_type": "linear",
                       "environment_complexity": "simple", "max_speed": 25.0, "lidar_fps": 15},
    "parking_detailed": {"duration": 30.0, "trajectory_type": "circular",
                         "environment_complexity": "medium", "max_speed": 5.0, "lidar_fps": 20},
}
FRAMES = {"urban_complex": [0, 1, 2, 599, 1199], "parking_detailed": [0, 300], "highway_simple": [0, 1]}


def make_lmc(lmc):
    out = {}
    for name, cfg in SCENARIOS.items():
        sim = lmc.LiDARMotionSimulator(dict(cfg))
        with contextlib.redirect_stdout(io.StringIO()):
            res = sim.run_simulation()
        tr = res["trajectory"]
        np.savez_compressed(os.path.join(HERE, f"lmc_traj_{name}.npz"), time=tr["time"],
                            position=tr["position"], velocity=tr["velocity"],
                            orientation=tr["orientation"], position_gps=tr["position_gps"],
                            orientation_imu=tr["orientation_imu"], acceleration=tr["acceleration"])
        frames = list(FRAMES[name])
        if name == "highway_simple":  # add one empty frame (845 of 900 are empty)
            empty = [s["frame_id"] for s in res["raw_scans"] if len(s["points_local"]) == 0]
            frames.append(empty[0])
        for fid in frames:
            scan = res["raw_scans"][fid]
            pos = scan["sensor_pose"]["position"]
            idx = int(np.flatnonzero(np.all(tr["position_gps"] == pos, axis=1))[0])
            key = f"{name}/{fid}"
            out[key + "/points_local"] = np.asarray(scan["points_local"], dtype=np.float64).reshape(-1, 4)
            out[key + "/aligned"] = np.asarray(res["aligned_pointclouds"][fid], dtype=np.float64).reshape(-1, 4)
            out[key + "/pose_idx"] = np.int64(idx)
            out[key + "/position"] = np.asarray(pos)
            out[key + "/rpy"] = np.asarray(scan["sensor_pose"]["orientation"])
            out[key + "/t_frame"] = np.float64(scan["timestamp"])
        out[name + "/n_frames"] = np.int64(len(res["raw_scans"]))
        out[name + "/frame_counts"] = np.array([len(s["points_local"]) for s in res["raw_scans"]], np.int64)
        print(f"{name}: {len(res['raw_scans'])} frames, fixtures for {frames}")
    np.savez_compressed(os.path.join(HERE, "lmc_frames.npz"), **out)


def make_env(lmc):
    """The scene each scenario scans and the global RNG state right before the reference's frame
    loop (LMC:802): run_simulation draws trajectory noise (LMC:785) and the environment (LMC:789)
    first, so replaying those steps from a fresh seed-42 construction reproduces both."""
    for name, cfg in SCENARIOS.items():
        sim = lmc.LiDARMotionSimulator(dict(cfg))
        sim.add_sensor_noise(sim.generate_trajectory())
        env = sim.generate_environment_pointcloud()
        kind, keys, pos, has_gauss, cached = np.random.get_state()
        np.savez_compressed(os.path.join(HERE, f"lmc_env_{name}.npz"), environment=env,
                            rng_keys=keys, rng_pos=np.int64(pos), rng_has_gauss=np.int64(has_gauss),
                            rng_cached=np.float64(cached))


def make_kat(lmc):
    rng = np.random.default_rng(7)
    sim = lmc.LiDARMotionSimulator()
    pts = np.column_stack([rng.uniform(-80, 80, (64, 3)), rng.uniform(0, 1, 64)])
    cases = [
        ([0.0, 0.0, 0.0], [0.0, 0.0, 0.0]),
        ([12.5, -3.0, 1.5], [0.0, 0.0, 0.0]),           # zero rotation => pure translation
        ([0.0, 0.0, 0.0], [0.0, 0.0, np.pi / 2]),       # yaw = pi/2 permutes x/y
        ([1500.0, 4.9, 0.0], [0.05, -0.02, 3.1]),       # highway-scale translation, near yaw wrap
        ([-30.0, 29.0, 1.5], [-0.08, 0.01, -3.13]),
        ([5.0, 5.0, 5.0], [0.7, -0.4, 2.0]),
    ]
    out = {"points": pts}
    for i, (t, r) in enumerate(cases):
        out[f"t{i}"] = np.array(t)
        out[f"r{i}"] = np.array(r)
        out[f"out{i}"] = sim.transform_pointcloud(pts, {"translation": np.array(t), "rotation": np.array(r)})
        # every point as a one-point frame: numpy's matrix-vector product sums in another order
        out[f"one{i}"] = np.vstack([sim.transform_pointcloud(pts[j:j + 1], {"translation": np.array(t),
                                                                              "rotation": np.array(r)})
                                    for j in range(len(pts))])
    out["empty_out"] = sim.transform_pointcloud(np.zeros((0, 4)), {"translation": np.zeros(3), "rotation": np.zeros(3)})
    # one frame above the zero-copy size (the library's DMA row pipeline path), highway-scale pose
    # (points regenerated by the test from this seed; the output's sha256 and every 1000th row kept)
    import hashlib
    brng = np.random.default_rng(2024)
    big = np.column_stack([brng.uniform(-90, 90, (40_000, 3)), brng.uniform(0, 1, 40_000)])
    bo = sim.transform_pointcloud(big, {"translation": np.array(cases[3][0]), "rotation": np.array(cases[3][1])})
    out["big/sha256"] = np.frombuffer(hashlib.sha256(np.ascontiguousarray(bo).tobytes()).digest(), np.uint8)
    out["big/rows"] = bo[::1000]
    out["n_cases"] = np.int64(len(cases))
    np.savez_compressed(os.path.join(HERE, "lmc_kat.npz"), **out)


def make_config(lmc):
    sim = lmc.LiDARMotionSimulator()
    bad = [
        {"duration": "60"}, {"lidar_fps": 0}, {"lidar_fps": -5}, {"duration": 0.0},
        {"max_speed": -1.0}, {"range_max": 1.0, "range_min": 2.0}, {"range_max": 2.0, "range_min": 2.0},
        {"points_per_frame": None}, {"range_min": 5.0},
    ]
    errors = []
    for cfg in bad:
        try:
            lmc.LiDARMotionSimulator(cfg)
            errors.append({"config": cfg, "error": None, "message": None})
        except Exception as e:  # noqa: BLE001
            errors.append({"config": cfg, "error": type(e).__name__, "message": str(e)})
    sim2 = lmc.LiDARMotionSimulator({"trajectory_type": "spiral"})
    try:
        sim2.generate_trajectory()
        unk = {"error": None}
    except Exception as e:  # noqa: BLE001
        unk = {"error": type(e).__name__, "message": str(e)}
    with open(os.path.join(HERE, "lmc_config.json"), "w") as f:
        json.dump({"defaults": sim.default_config(), "errors": errors, "unknown_trajectory": unk}, f, indent=1)


def make_pathb(csim):
    cfg = dict(csim.DEFAULT_CONFIG)
    with contextlib.redirect_stderr(io.StringIO()):
        traj = csim.TrajectoryGenerator("figure_eight", 42).generate_trajectory(duration=10.0, max_speed=12.0)
        imu = csim.IMUSimulator(cfg).simulate_imu_data(traj, 10.0)
        comp = csim.MotionCompensator(cfg)
    rng = np.random.default_rng(11)

    def imu_arr(lst):
        return (np.array([s.timestamp for s in lst], np.int64),
                np.array([[s.gyro_x, s.gyro_y, s.gyro_z, s.accel_x, s.accel_y, s.accel_z] for s in lst]).reshape(-1, 6))

    def run(case, imu_list, frame_start, ts):
        n = len(ts)
        xyz = np.column_stack([rng.uniform(0.05, 90, n), rng.uniform(-60, 60, n), rng.uniform(-70, 70, n)])
        inten = rng.integers(0, 256, n)
        pts = [csim.LiDARPoint(x=float(xyz[i, 0]), y=float(xyz[i, 1]), z=float(xyz[i, 2]), intensity=int(inten[i]),
                               timestamp=int(ts[i]), ring=i % 16, tag=i % 2) for i in range(n)]
        out = comp.compensate_point_cloud(pts, imu_list, int(frame_start), 100_000_000)
        its, ig = imu_arr(imu_list)
        return {f"{case}/imu_ts": its, f"{case}/imu_gyro": ig[:, :3], f"{case}/imu_accel": ig[:, 3:],
                f"{case}/frame_start": np.int64(frame_start), f"{case}/xyz": xyz,
                f"{case}/intensity": inten.astype(np.int64), f"{case}/ts": np.asarray(ts, np.int64),
                f"{case}/ring": np.arange(n) % 16, f"{case}/tag": np.arange(n) % 2,
                f"{case}/out_xyz": np.array([[p.x, p.y, p.z] for p in out]),
                f"{case}/out_meta": np.array([[p.intensity, p.timestamp, p.ring, p.tag] for p in out], np.int64)}

    out = {}
    # 1000 returns spread over a frame at 1.2 s (CSIM:1048 spacing), some on IMU sample times
    fs = 1_200_000_000
    out.update(run("mid", imu, fs, fs + np.arange(1000) * 1000 * 100))
    # frame starting before the first IMU sample (negative timestamps -> first sample used)
    fs = -3_000_000
    out.update(run("before", imu, fs, fs + np.arange(400) * 25_000))
    # frame running past the last IMU sample (9.995 s)
    fs = 9_950_000_000
    out.update(run("after", imu, fs, fs + np.arange(400) * 250_000))
    # duplicate timestamp pair: sample 300 repeated with different gyro values
    dup = list(imu[:301]) + [csim.IMUData(imu[300].timestamp, imu[300].gyro_x + 0.5, imu[300].gyro_y - 0.25,
                                          imu[300].gyro_z + 1.0, 0.0, 0.0, 9.81)] + list(imu[301:])
    t300 = imu[300].timestamp
    fs = t300 - 40_000_000
    ts = np.sort(np.concatenate([fs + np.arange(200) * 400_000, [t300, t300, t300 - 1, t300 + 1]]))
    out.update(run("dup", dup, fs, ts))
    # yaw-wrap gyro spike region: the Euler-difference gyro of CSIM:1214-1217 jumps at +-pi
    ts_all, g_all = imu_arr(imu)
    spike = int(np.argmax(np.abs(g_all[:, 2])))
    fs = int(ts_all[max(spike - 10, 0)])
    out.update(run("spike", imu, fs, fs + np.arange(500) * 200_000))
    out["spike/max_gyro"] = np.float64(np.abs(g_all[:, 2]).max())
    # empty IMU list -> points unchanged (CSIM:1439-1440)
    out.update(run("noimu", [], 0, np.arange(50) * 1000))
    np.savez_compressed(os.path.join(HERE, "csim_pathb.npz"), **out)
    print("path B: IMU samples", len(imu), "max |gyro_z|", out["spike/max_gyro"])


def make_slerp(lmc):
    from scipy.spatial.transform import Rotation, Slerp
    sim = lmc.LiDARMotionSimulator(dict(SCENARIOS["parking_detailed"]))
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    yaw = tr["orientation_imu"][:, 2]
    wrap = int(np.flatnonzero(np.abs(np.diff(yaw)) > np.pi)[0])   # yaw jumps +-pi between wrap, wrap+1
    t_lo, t_hi = tr["time"][wrap - 1], tr["time"][wrap + 2]
    rng = np.random.default_rng(5)
    n = 1000
    tq = np.sort(rng.uniform(t_lo, t_hi, n))
    tq[:3] = tr["time"][wrap - 1:wrap + 2]                         # exact sample times
    rots = Rotation.from_euler("xyz", tr["orientation_imu"])
    R = Slerp(tr["time"], rots)(tq)
    pos = np.stack([np.interp(tq, tr["time"], tr["position_gps"][:, j]) for j in range(3)], axis=1)
    xyz = np.column_stack([rng.uniform(0.05, 90, n), rng.uniform(-60, 60, n), rng.uniform(-70, 70, n)])
    out = R.apply(xyz) + pos
    np.savez_compressed(os.path.join(HERE, "slerp.npz"), time=tr["time"], position_gps=tr["position_gps"],
                        orientation_imu=tr["orientation_imu"], tq=tq, xyz=xyz, out=out, wrap=np.int64(wrap))


def make_synth():
    from oracle import synth
    x, y, z, i, t = synth.synth_frame(100_000, 0, 1000)
    np.savez_compressed(os.path.join(HERE, "synth.npz"), x=x[:4096], y=y[:4096], z=z[:4096], i=i[:4096],
                        t=t[:4096], sums=np.array([x.astype(np.float64).sum(), y.astype(np.float64).sum(),
                                                   z.astype(np.float64).sum(), i.astype(np.float64).sum(),
                                                   t.astype(np.float64).sum()]))


PCD_TRICKY = [0.0078125, -0.0078125, -0.0, 0.0, -1e-9, 1e-9, 5e-7, -5e-7, 1.5e-6, 2.5e-6, 1e-7, 1 / 3, -2 / 3,
              999999.9999995, 123456.7890125, 0.0000015, 1e20, -3.4e30, 2.0 ** 53 + 2, 0.1, 0.2, 0.3, 1e-300,
              4.0000005, 12.3456785, 7.5e-7, 2.5e-7, 99.9999995, -99.9999995, 1e15 + 0.5, 65504.0]


def make_codecs(lmc):
    """LVX v1.1 packer (LMC:24-272) and ASCII PCD writer (LMC:932-948) outputs, byte for byte."""
    import tempfile
    rng = np.random.default_rng(77)
    w = lmc.LivoxLVXWriter()
    out = {}

    def frame(n, ncol=4, scale=40.0):
        p = rng.normal(0, scale, (n, 3))
        cols = [p] + ([rng.uniform(-0.2, 1.2, (n, 1))] if ncol > 3 else [])
        return np.hstack(cols)

    clip = frame(96)
    clip[:8, 0] = [3e6, -3e6, 1.0005, -0.0009, 2147483.6475, -2147483.6485, 1e300, -1e300]
    clip[:6, 3] = [1.5, -0.5, 0.999999, 1.0, 0.0, 254.5 / 255]
    frames = [
        {"frame_id": 0, "timestamp": 0.0, "points": frame(97)},
        {"frame_id": 1, "timestamp": 0.1, "points": np.zeros((0, 4))},
        {"frame_id": 2, "timestamp": 0.2, "points": clip},
        {"frame_id": 7, "timestamp": 12.345678912, "points": frame(1)},
        {"frame_id": 8, "timestamp": 119.9, "points": frame(300, ncol=3)},
        {"frame_id": 9, "timestamp": 120.0, "points": frame(1000, scale=0.01)},
    ]
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, "t.lvx")
        with contextlib.redirect_stdout(io.StringIO()):
            ok = w.write_compatible_lvx(fn, frames)
        assert ok
        with open(fn, "rb") as fh:
            out["lvx/bytes"] = np.frombuffer(fh.read(), np.uint8)
        for i, fr in enumerate(frames):
            out[f"lvx/{i}/points"] = fr["points"]
            out[f"lvx/{i}/frame_id"] = np.int64(fr["frame_id"])
            out[f"lvx/{i}/timestamp"] = np.float64(fr["timestamp"])
        out["lvx/n_frames"] = np.int64(len(frames))
        # a NaN coordinate: the writer's int() raises inside its try -> returns False
        bad = [{"frame_id": 0, "timestamp": 0.0, "points": np.array([[np.nan, 0, 0, 0.5]])}]
        with contextlib.redirect_stdout(io.StringIO()):
            out["lvx/nan_ok"] = np.bool_(w.write_compatible_lvx(os.path.join(d, "bad.lvx"), bad))

        sim = lmc.LiDARMotionSimulator()
        t = np.array(PCD_TRICKY, np.float64)
        n4 = (len(t) + 3) // 4 * 4
        tricky = np.resize(t, n4).reshape(-1, 4)
        specials = np.array([[np.inf, -np.inf, np.nan, 1.0], [-np.nan, 0.5, 2.0, -np.inf]])
        cases = {"tricky": tricky, "specials": specials, "random": frame(2000, scale=60.0),
                 "f32": frame(500).astype(np.float32).astype(np.float64), "empty": np.zeros((0, 4)),
                 "wide": np.hstack([frame(10), np.full((10, 2), 9.0)])}
        for name, pts in cases.items():
            fn = os.path.join(d, f"{name}.pcd")
            sim.save_pcd(pts, fn)
            with open(fn, "rb") as fh:
                out[f"pcd/{name}/bytes"] = np.frombuffer(fh.read(), np.uint8)
            out[f"pcd/{name}/points"] = pts
    np.savez_compressed(os.path.join(HERE, "codecs.npz"), **out)


def make_coords(csim):
    """CoordinateTransformer (CSIM:153-233) and _transform_coordinates (CSIM:2107-2163)."""
    rng = np.random.default_rng(21)
    ct = csim.CoordinateTransformer()
    ct.set_transformation("sensor", "local", [10.0, -5.0, 2.0], [0.1, -0.2, 2.5])
    p3 = rng.normal(0, 30, (200, 3))
    p4 = np.column_stack([rng.normal(0, 30, (50, 3)), rng.uniform(0, 1, 50)])
    out = {"p3": p3, "p4": p4}
    with contextlib.redirect_stderr(io.StringIO()):
        for a, b in [("sensor", "vehicle"), ("sensor", "local"), ("local", "sensor"), ("sensor", "sensor"),
                     ("vehicle", "sensor")]:
            out[f"tp/{a}/{b}"] = ct.transform_points(p3, a, b)
        out["tp4/sensor/local"] = ct.transform_points(p4, "sensor", "local")
        out["T/sensor/local"] = ct.transformations[("sensor", "local")]
        out["T/local/sensor"] = ct.transformations[("local", "sensor")]

        class Stub:
            coordinate_transformer = ct

            def _find_closest_gps_sample(self, gps, ts):
                return csim.LiDARMotionSimulator._find_closest_gps_sample(self, gps, ts)

        counts = [40, 0, 7]
        frames = []
        for i, n in enumerate(counts):
            xyz = rng.normal(0, 20, (n, 3))
            pts = [csim.LiDARPoint(x=float(x), y=float(y), z=float(z), intensity=int(k % 256),
                                   timestamp=int(1_000_000 * k), ring=0, tag=0) for k, (x, y, z) in enumerate(xyz)]
            frames.append({"frame_id": i, "timestamp": int(i * 100_000_000), "points": pts})
            out[f"tc/in/{i}"] = xyz.reshape(n, 3)
        gps = [csim.GPSData(timestamp=0, latitude=40.0, longitude=-74.0, altitude=10.0, velocity_x=0.0,
                            velocity_y=0.0, velocity_z=0.0, heading=0.0)]
        for target in ("vehicle", "local", "utm"):
            res = csim.LiDARMotionSimulator._transform_coordinates(Stub(), frames, target, gps)
            for i, fr in enumerate(res):
                out[f"tc/{target}/{i}"] = np.array([[p.x, p.y, p.z] for p in fr["points"]]).reshape(-1, 3)
                out[f"tc/{target}/{i}/meta"] = np.array([[p.intensity, p.timestamp] for p in fr["points"]],
                                                        np.int64).reshape(-1, 2)
                assert fr["coordinate_system"] == target
        out["tc/n_frames"] = np.int64(len(counts))
        out["utm_available"] = np.bool_(csim.UTM_AVAILABLE)
        # a UTM-scale translation (easting / northing ~ 5e5 / 4.4e6 m): float32 would quantise it to 0.5 m
        ct.set_transformation("sensor", "utm_grid", [512345.678, 4431234.567, 12.5], [0.01, -0.02, 1.2])
        pb = rng.normal(0, 40, (300, 3))
        out["big/p3"] = pb
        out["big/T"] = ct.transformations[("sensor", "utm_grid")]
        out["big/T_inv"] = ct.transformations[("utm_grid", "sensor")]
        out["big/fwd"] = ct.transform_points(pb, "sensor", "utm_grid")
        out["big/back"] = ct.transform_points(out["big/fwd"], "utm_grid", "sensor")
    np.savez_compressed(os.path.join(HERE, "coords.npz"), **out)


def make_save_results(lmc):
    """LMC:860-931 on a small results dict: every file save_results writes, byte for byte."""
    import tempfile
    rng = np.random.default_rng(31)
    n_frames = 4
    sizes = [50, 0, 130, 7]
    tr = {"time": np.linspace(0, 1, 6), "position": rng.normal(0, 10, (6, 3)),
          "position_gps": rng.normal(0, 10, (6, 3))}
    raw, aligned, motion = [], [], []
    for i, n in enumerate(sizes):
        loc = np.column_stack([rng.normal(0, 30, (n, 3)), rng.uniform(0, 1, n)]).reshape(n, 4)
        al = np.column_stack([rng.normal(0, 300, (n, 3)), loc[:, 3]]).reshape(n, 4)
        pose = {"position": tr["position_gps"][i], "orientation": rng.normal(0, 0.1, 3),
                "velocity": rng.normal(0, 5, 3)}
        raw.append({"frame_id": i, "timestamp": 0.1 * i, "points_local": loc, "sensor_pose": pose})
        aligned.append(al)
        motion.append({"frame_id": i, "timestamp": 0.1 * i, "gps_lat": 40.0 + i * 1e-5, "gps_lon": -74.0,
                       "gps_alt": 1.5, "imu_roll": 0.01 * i, "imu_pitch": -0.02, "imu_yaw": 1.0 + i,
                       "vel_x": 3.0, "vel_y": 0.5 * i, "vel_z": 0.0})
    results = {"raw_scans": raw, "aligned_pointclouds": aligned, "motion_data": motion, "trajectory": tr}
    out = {}
    for tag, res in (("gap", results),
                     ("full", dict(results, aligned_pointclouds=[a for a in aligned if len(a)],
                                   raw_scans=[s for s in raw if len(s["points_local"])]))):
        sim = lmc.LiDARMotionSimulator()
        with tempfile.TemporaryDirectory() as d, contextlib.redirect_stdout(io.StringIO()):
            sim.save_results(res, d)
            for root, _, files in os.walk(d):
                for fn in sorted(files):
                    p = os.path.join(root, fn)
                    with open(p, "rb") as fh:
                        out[f"{tag}/{os.path.relpath(p, d)}"] = np.frombuffer(fh.read(), np.uint8)
        for i, s in enumerate(res["raw_scans"]):
            out[f"{tag}/in/raw/{i}"] = s["points_local"]
            out[f"{tag}/in/frame_id/{i}"] = np.int64(s["frame_id"])
        for i, a in enumerate(res["aligned_pointclouds"]):
            out[f"{tag}/in/aligned/{i}"] = a
    for k in ("time", "position", "position_gps"):
        out[f"in/trajectory/{k}"] = tr[k]
    out["in/motion"] = np.array([[m[c] for c in motion[0]] for m in motion], np.float64)
    out["in/motion_cols"] = np.array(list(motion[0]))
    out["in/n_frames"] = np.int64(n_frames)
    np.savez_compressed(os.path.join(HERE, "save_results.npz"), **out)


def make_run_files(lmc):
    """Digest of every file the reference writes for a whole scenario (LMC:1176-1233 minus the
    plots and report): run_simulation -> save_results into a temp dir."""
    import hashlib
    import shutil
    import tempfile
    out = {}
    for name, cfg in SCENARIOS.items():
        sim = lmc.LiDARMotionSimulator(dict(cfg))
        with contextlib.redirect_stdout(io.StringIO()):
            res = sim.run_simulation()
        e = np.load(os.path.join(HERE, f"lmc_env_{name}.npz"))
        assert np.array_equal(e["environment"], res["environment"]), name
        d = tempfile.mkdtemp()
        try:
            log = io.StringIO()
            with contextlib.redirect_stdout(log):
                sim.save_results(res, d)
            files = {}
            for root, _, fs in os.walk(d):
                for fn in sorted(fs):
                    p = os.path.join(root, fn)
                    with open(p, "rb") as fh:
                        data = fh.read()
                    files[os.path.relpath(p, d)] = [len(data), hashlib.sha256(data).hexdigest()]
            out[name] = {"files": files, "log": log.getvalue().replace(d, "<out>"),
                         "frame_counts": [int(len(s["points_local"])) for s in res["raw_scans"]]}
        finally:
            shutil.rmtree(d)
        print(f"{name}: {len(out[name]['files'])} files, {sum(v[0] for v in out[name]['files'].values())} bytes")
    with open(os.path.join(HERE, "lmc_run_files.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)


def main():
    lmc, csim = import_reference()
    one = {"run_files": lambda: make_run_files(lmc), "coords": lambda: make_coords(csim), "kat": lambda: make_kat(lmc)}
    if sys.argv[1:2] and sys.argv[1] in one:   # one fixture only (the others are unchanged by it)
        one[sys.argv[1]]()
        return
    make_save_results(lmc)
    make_coords(csim)
    make_codecs(lmc)
    make_lmc(lmc)
    make_env(lmc)
    make_kat(lmc)
    make_config(lmc)
    make_pathb(csim)
    make_slerp(lmc)
    make_synth()
    make_run_files(lmc)
    for f in sorted(os.listdir(HERE)):
        print(f"{f:24s} {os.path.getsize(os.path.join(HERE, f)):>9d} B")


if __name__ == "__main__":
    main()
