"""CPU restatement of the reference's motion-compensation path (float64, numpy).

TEST INFRASTRUCTURE ONLY.  This module is the parity oracle: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker / the timed CPU baseline.  The product path
(``livox-motion-compensation-sim_amd``) never imports it and fails loudly when
its HIP library is missing.

Parity status: PINNED.  Every function below is checked in ``tests/test_oracle_golden.py``
against golden vectors produced by running the reference itself in the build
container (``tests/golden/make_golden.py``; reference imported with a stub ``laspy``
module, which the reference uses only in ``save_las``, LMC:950-963).

Abbreviations: LMC = lidar_motion_compensation.py, CSIM = livox_mid70_complete_simulator.py
(both under the reference root).  Third-party arithmetic on the path: scipy
``Rotation.from_euler('xyz', ...)`` (LMC:11, 774), scipy 1.15.3 in this image; the
reference pins no versions.  ``from_euler('xyz')`` is extrinsic x->y->z, i.e.
R = Rz(yaw) Ry(pitch) Rx(roll); restated explicitly in ``euler_xyz_matrix``.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "euler_xyz_matrix", "euler_xyz_quat", "select_pose_index", "transform_pointcloud", "transform_pointcloud_ref_ops",
    "align_frames", "merge_aligned", "scan_environment", "imu_interpolate_gyro", "compensate_arrays",
    "compensate_point_cloud_loop", "slerp_pose", "deskew_pose_slerp",
]


# ----------------------------------------------------------------------------------------------
# Path A: per-frame global alignment (LMC:772-776, 802-832, 887-889)
# ----------------------------------------------------------------------------------------------
def euler_xyz_matrix(rpy) -> np.ndarray:
    """R = Rz(yaw) @ Ry(pitch) @ Rx(roll) == Rotation.from_euler('xyz', rpy).as_matrix() (LMC:774).

    Accepts (3,) or (n,3); returns (3,3) or (n,3,3).  Cross-checked against CSIM:187-212's
    explicit builder and scipy in tests.
    """
    rpy = np.asarray(rpy, dtype=np.float64)
    r, p, y = rpy[..., 0], rpy[..., 1], rpy[..., 2]
    sr, cr, sp, cp, sy, cy = np.sin(r), np.cos(r), np.sin(p), np.cos(p), np.sin(y), np.cos(y)
    R = np.empty(rpy.shape[:-1] + (3, 3))
    R[..., 0, 0] = cy * cp
    R[..., 0, 1] = cy * sp * sr - sy * cr
    R[..., 0, 2] = cy * sp * cr + sy * sr
    R[..., 1, 0] = sy * cp
    R[..., 1, 1] = sy * sp * sr + cy * cr
    R[..., 1, 2] = sy * sp * cr - cy * sr
    R[..., 2, 0] = -sp
    R[..., 2, 1] = cp * sr
    R[..., 2, 2] = cp * cr
    return R


def euler_xyz_quat(rpy) -> np.ndarray:
    """Unit quaternion (x, y, z, w) of euler_xyz_matrix(rpy) (q = qz * qy * qx)."""
    rpy = np.asarray(rpy, dtype=np.float64)
    h = 0.5 * rpy
    sr, cr = np.sin(h[..., 0]), np.cos(h[..., 0])
    sp, cp = np.sin(h[..., 1]), np.cos(h[..., 1])
    sy, cy = np.sin(h[..., 2]), np.cos(h[..., 2])
    return np.stack([sr * cp * cy - cr * sp * sy,
                     cr * sp * cy + sr * cp * sy,
                     cr * cp * sy - sr * sp * cy,
                     cr * cp * cy + sr * sp * sy], axis=-1)


def select_pose_index(time: np.ndarray, t_frame) -> np.ndarray:
    """Zero-order-hold 'next-or-equal' pose: clamp(searchsorted(time, t, 'left'), 0, T-1) (LMC:804-806)."""
    idx = np.searchsorted(np.asarray(time, dtype=np.float64), t_frame)
    return np.clip(idx, 0, len(time) - 1)


def transform_pointcloud(points, transformation) -> np.ndarray:
    """LMC:772-776: p' = R(rotation) p + translation; intensity column passed through.

    Same op sequence as the reference: R @ P[:, :3].T, .T + t, column_stack.
    """
    points = np.asarray(points)
    R = euler_xyz_matrix(np.asarray(transformation["rotation"], dtype=np.float64))
    transformed = (R @ points[:, :3].T).T + np.asarray(transformation["translation"], dtype=np.float64)
    return np.column_stack([transformed, points[:, 3]])


def transform_pointcloud_ref_ops(points, transformation) -> np.ndarray:
    """LMC:772-776 as the reference executes it, op for op: scipy ``Rotation.from_euler('xyz',
    rotation).as_matrix()`` (LMC:774), ``R @ points[:, :3].T`` (775), ``.T + translation`` (775),
    ``np.column_stack`` with the intensity column (776).  Used as bench.py's frame-mode CPU
    baseline (the reference's own per-frame cost); numerically equal to transform_pointcloud."""
    from scipy.spatial.transform import Rotation
    R = Rotation.from_euler("xyz", transformation["rotation"]).as_matrix()
    transformed = (R @ points[:, :3].T).T + transformation["translation"]
    return np.column_stack([transformed, points[:, 3]])


def align_frames(scans, trajectory, times) -> list:
    """The hot loop of run_simulation (LMC:802-832) minus scanning: per frame, select the pose
    (LMC:804-812) and transform the frame's local scan (LMC:826-831)."""
    out = []
    idx = select_pose_index(trajectory["time"], np.asarray(times))
    for scan, k in zip(scans, idx):
        out.append(transform_pointcloud(scan, {"translation": trajectory["position_gps"][k],
                                               "rotation": trajectory["orientation_imu"][k]}))
    return out


def scan_environment(environment, sensor_pose, config, rng=np.random) -> np.ndarray:
    """LMC:701-770: local scan of the scene from a pose.  Range prefilter on the world distance
    (709-723), R^T (p - t) into the sensor frame (726-728), FOV mask on atan2 / asin in degrees and
    range_min (735-745), systematic subsample to points_per_frame (754-762), N(0, range_noise)
    added to the kept points from the global RNG (765-768); returns (n, 4) [x, y, z, intensity]."""
    env = np.asarray(environment, dtype=np.float64)
    pos = np.asarray(sensor_pose["position"], dtype=np.float64)
    d2 = np.sum((env[:, :3] - pos) ** 2, axis=1)
    keep = d2 <= config["range_max"] ** 2
    if not np.any(keep):
        return np.zeros((0, 4))
    envf = env[keep]
    Rm = euler_xyz_matrix(np.asarray(sensor_pose["orientation"], dtype=np.float64))
    loc = (Rm.T @ (envf[:, :3] - pos).T).T
    rng_ = np.sqrt(d2[keep])
    az = np.arctan2(loc[:, 1], loc[:, 0]) * 180 / np.pi
    el = np.arcsin(np.clip(loc[:, 2] / np.maximum(rng_, 1e-6), -1, 1)) * 180 / np.pi
    fov = ((np.abs(az) <= config["fov_horizontal"] / 2) & (np.abs(el) <= config["fov_vertical"] / 2)
           & (rng_ >= config["range_min"]))
    if not np.any(fov):
        return np.zeros((0, 4))
    pts = loc[fov]
    inten = envf[fov, 3]
    n, cap = len(pts), config["points_per_frame"]
    if n > cap:
        sel = np.arange(0, n, n // cap)[:cap]
        pts, inten = pts[sel], inten[sel]
    if config["lidar_range_noise"] > 0:
        pts = pts + rng.normal(0, config["lidar_range_noise"], pts.shape)
    return np.column_stack([pts, inten])


def merge_aligned(aligned) -> np.ndarray:
    """LMC:887-889: frame-ordered np.vstack (the reference skips it if any frame is empty)."""
    if not aligned:
        return np.zeros((0, 4))
    return np.vstack(aligned)


# ----------------------------------------------------------------------------------------------
# Path B: per-point IMU deskew (CSIM:1435-1536)
# ----------------------------------------------------------------------------------------------
def imu_interpolate_gyro(imu_ts: np.ndarray, gyro: np.ndarray, t: np.ndarray) -> np.ndarray:
    """Vectorised _interpolate_imu_data (CSIM:1482-1516) for sorted IMU timestamps.

    before = last sample with ts <= t, after = first sample with ts > t; only one side present
    -> that sample (CSIM:1496-1497); else gyro_b + alpha*(gyro_a - gyro_b),
    alpha = (t - ts_b) / (ts_a - ts_b) (CSIM:1504-1511).
    """
    imu_ts = np.asarray(imu_ts, dtype=np.int64)
    gyro = np.asarray(gyro, dtype=np.float64)
    t = np.asarray(t, dtype=np.int64)
    c = np.searchsorted(imu_ts, t, side="right")       # samples with ts <= t
    M = len(imu_ts)
    out = np.empty((len(t), 3))
    first = c == 0
    last = c == M
    mid = ~(first | last)
    out[first] = gyro[0]
    out[last] = gyro[M - 1]
    b = c[mid] - 1
    a = c[mid]
    alpha = (t[mid] - imu_ts[b]) / (imu_ts[a] - imu_ts[b])
    out[mid] = gyro[b] + alpha[:, None] * (gyro[a] - gyro[b])
    return out


def compensate_arrays(xyz, t_ns, frame_start_ns: int, imu_ts, gyro) -> np.ndarray:
    """compensate_point_cloud (CSIM:1435-1480) on arrays: theta = w(t)*dt, p' = R_xyz(theta)^T p,
    dt = (t - frame_start)*1e-9 (CSIM:1454-1465).  Rotation only, no translation.
    Empty IMU -> points unchanged (CSIM:1439-1440)."""
    xyz = np.asarray(xyz, dtype=np.float64)
    if len(imu_ts) == 0:
        return xyz.copy()
    t_ns = np.asarray(t_ns, dtype=np.int64)
    w = imu_interpolate_gyro(imu_ts, gyro, t_ns)
    dt = (t_ns - int(frame_start_ns)) * 1e-9
    theta = w * dt[:, None]
    R = euler_xyz_matrix(theta)                       # Rz Ry Rx of theta
    return np.einsum("nji,nj->ni", R, xyz)            # R^T p == Rx(-a) Ry(-b) Rz(-c) p (CSIM:1518-1536)


def compensate_point_cloud_loop(points, imu, frame_start_ns: int):
    """Literal per-point restatement of CSIM:1435-1536 (pure Python; small cases only).

    points: list of (x, y, z, intensity, timestamp, ring, tag); imu: list of
    (timestamp, gx, gy, gz, ax, ay, az).  Returns the same tuple layout.
    """
    if not imu:
        return list(points)
    out = []
    for (x, y, z, inten, ts, ring, tag) in points:
        before = after = None
        for s in imu:                                  # CSIM:1489-1494
            if s[0] <= ts:
                before = s
            elif s[0] > ts and after is None:
                after = s
                break
        if before is None or after is None:
            smp = before or after
            g = smp[1:4]
        else:
            td = after[0] - before[0]
            if td == 0:
                g = before[1:4]
            else:
                al = (ts - before[0]) / td
                g = tuple(before[j] + al * (after[j] - before[j]) for j in (1, 2, 3))
        dt = (ts - frame_start_ns) * 1e-9
        rx, ry, rz = (g[0] * dt, g[1] * dt, g[2] * dt)
        Rx = np.array([[1, 0, 0], [0, np.cos(-rx), -np.sin(-rx)], [0, np.sin(-rx), np.cos(-rx)]])
        Ry = np.array([[np.cos(-ry), 0, np.sin(-ry)], [0, 1, 0], [-np.sin(-ry), 0, np.cos(-ry)]])
        Rz = np.array([[np.cos(-rz), -np.sin(-rz), 0], [np.sin(-rz), np.cos(-rz), 0], [0, 0, 1]])
        v = Rx @ Ry @ Rz @ np.array([x, y, z])
        out.append((v[0], v[1], v[2], inten, ts, ring, tag))
    return out


# ----------------------------------------------------------------------------------------------
# Build-added per-point pose interpolation
# ----------------------------------------------------------------------------------------------
def slerp_pose(time, position, rpy, t_query):
    """Pose at arbitrary times: quaternion SLERP (shortest arc) + position LERP between the
    bracketing samples; clamped to the first/last sample outside the table.

    Segment k = clip(searchsorted(time, t, 'right') - 1, 0, T-2); alpha = clip((t - t_k)/dt, 0, 1).
    At t == time[j] this is exactly sample j, so it reduces to Path A's pose at sample times.
    Returns (R (n,3,3), p (n,3)).  Cross-checked against scipy's Slerp in tests.
    """
    time = np.asarray(time, dtype=np.float64)
    position = np.asarray(position, dtype=np.float64)
    t_query = np.asarray(t_query, dtype=np.float64)
    T = len(time)
    q = euler_xyz_quat(rpy)
    if T == 1:
        n = len(t_query)
        return (np.broadcast_to(euler_xyz_matrix(rpy[0]), (n, 3, 3)).copy(),
                np.broadcast_to(position[0], (n, 3)).copy())
    k = np.clip(np.searchsorted(time, t_query, side="right") - 1, 0, T - 2)
    dt = time[k + 1] - time[k]
    with np.errstate(divide="ignore", invalid="ignore"):
        al = np.where(dt > 0, (t_query - time[k]) / np.where(dt > 0, dt, 1.0), 0.0)
    al = np.clip(al, 0.0, 1.0)
    q0 = q[k]
    q1 = q[k + 1].copy()
    d = np.sum(q0 * q1, axis=1)
    neg = d < 0
    q1[neg] = -q1[neg]
    d = np.minimum(np.abs(d), 1.0)
    th = np.arccos(d)
    small = th < 1e-6
    with np.errstate(divide="ignore", invalid="ignore"):
        s1 = np.where(small, al, np.sin(al * th) / np.where(small, 1.0, np.sin(th)))
        s0 = np.where(small, 1.0 - al, np.sin((1.0 - al) * th) / np.where(small, 1.0, np.sin(th)))
    qi = s0[:, None] * q0 + s1[:, None] * q1
    qi /= np.linalg.norm(qi, axis=1, keepdims=True)
    x, y, z, w = qi[:, 0], qi[:, 1], qi[:, 2], qi[:, 3]
    R = np.empty((len(qi), 3, 3))
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - z * w)
    R[:, 0, 2] = 2 * (x * z + y * w)
    R[:, 1, 0] = 2 * (x * y + z * w)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - x * w)
    R[:, 2, 0] = 2 * (x * z - y * w)
    R[:, 2, 1] = 2 * (y * z + x * w)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    p = position[k] + al[:, None] * (position[k + 1] - position[k])
    return R, p


def deskew_pose_slerp(xyz, t_ns, t_frame: float, trajectory) -> np.ndarray:
    """p' = R(q(t)) p + pos(t), t = t_frame + t_ns*1e-9 (the north-star per-point SE(3) deskew
    into the global frame)."""
    xyz = np.asarray(xyz, dtype=np.float64)
    tq = float(t_frame) + np.asarray(t_ns, dtype=np.int64) * 1e-9
    R, p = slerp_pose(trajectory["time"], trajectory["position_gps"], trajectory["orientation_imu"], tq)
    return np.einsum("nij,nj->ni", R, xyz) + p


# ----------------------------------------------------------------------------------------------
# CoordinateTransformer (CSIM:153-233)
# ----------------------------------------------------------------------------------------------
def create_transform_matrix(translation, rotation) -> np.ndarray:
    """CSIM:187-212: 4x4 [Rz(yaw) Ry(pitch) Rx(roll) | t]."""
    T = np.eye(4)
    T[:3, :3] = euler_xyz_matrix(np.asarray(rotation, dtype=np.float64))
    T[:3, 3] = translation
    return T


def transform_points_h(points, T) -> np.ndarray:
    """CSIM:214-233: (N,3) gets w = 1; any other width is used as homogeneous as it is."""
    p = np.asarray(points, dtype=np.float64)
    if p.shape[1] == 3:
        p = np.column_stack([p, np.ones(len(p))])
    return (np.asarray(T) @ p.T).T[:, :3]
