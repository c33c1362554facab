"""Drop-in ``MotionCompensator`` (CSIM:1426-1536) and the per-frame driver (CSIM:2086-2105).

``compensate_point_cloud`` keeps the reference signature and record types; the per-point work
(bracketing IMU samples, gyro LERP, theta = w*dt, p' = R_xyz(theta)^T p) runs on the GPU in float64
on the caller's float64 coordinates (``k_points_f64<2>``, mc_deskew_points_f64): no float32 staging,
so the result meets 1e-5 relative per coordinate on the reference's own data.
``compensate_arrays`` is the array form and ``apply_motion_compensation`` runs every frame of a run
in one launch.  Device-resident frames (``Batch``) go through ``Context.deskew(mode="imu")``, the
float32-column kernel ``k_deskew_points<2>`` the bench measures.

Contract difference from the reference, raised as ValueError rather than computed: IMU timestamps
must be non-decreasing (the reference's list scan, CSIM:1489-1494, assumes it).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List

import numpy as np

from .runtime import Context, default_context, deskew_points_f64


@dataclass
class IMUData:
    """CSIM:97-106 (200 Hz IMU record)."""
    timestamp: int
    gyro_x: float
    gyro_y: float
    gyro_z: float
    accel_x: float
    accel_y: float
    accel_z: float


@dataclass
class LiDARPoint:
    """CSIM:120-129 (one return)."""
    x: float
    y: float
    z: float
    intensity: int
    timestamp: int
    ring: int
    tag: int


def imu_to_arrays(imu_data) -> tuple:
    ts = np.fromiter((s.timestamp for s in imu_data), dtype=np.int64, count=len(imu_data))
    g = np.array([(s.gyro_x, s.gyro_y, s.gyro_z) for s in imu_data], dtype=np.float64).reshape(-1, 3)
    return ts, g


class MotionCompensator:
    """GPU-backed drop-in for livox_mid70_complete_simulator.MotionCompensator."""

    def __init__(self, config: Dict, *, context: Context | None = None):
        self.config = config
        self.enable_compensation = config.get("enable_motion_compensation", True)
        self._context = context

    @property
    def context(self) -> Context:
        if self._context is None:
            self._context = default_context()
        return self._context

    def _upload_imu(self, ts: np.ndarray, gyro: np.ndarray):
        """Arrays are rebuilt from the caller's data on every call (the reference reads the list
        each time, CSIM:1482-1516), so an in-place edit of any sample is always seen; the context
        skips only the device upload, and only for byte-equal contents."""
        if len(ts) > 1 and np.any(np.diff(ts) < 0):
            raise ValueError("IMU timestamps must be non-decreasing")
        self.context.set_imu(ts, gyro)

    # ---- reference signature (CSIM:1435) ---------------------------------------------------
    def compensate_point_cloud(self, points: List[LiDARPoint], imu_data: List[IMUData],
                               frame_start_time: int, frame_duration_ns: int) -> List[LiDARPoint]:
        """CSIM:1435-1480.  Returns ``points`` itself when disabled or without IMU data."""
        if not self.enable_compensation or not imu_data:
            return points
        if not points:
            return []
        self._imu_arrays(imu_data)          # built and uploaded once per call
        xyz = np.array([(p.x, p.y, p.z) for p in points], dtype=np.float64).reshape(-1, 3)
        t = np.fromiter((p.timestamp for p in points), dtype=np.int64, count=len(points))
        out = self._compensate_uploaded(xyz, t, frame_start_time)
        cls = type(points[0])
        return [cls(x=float(o[0]), y=float(o[1]), z=float(o[2]), intensity=p.intensity,
                    timestamp=p.timestamp, ring=p.ring, tag=p.tag) for o, p in zip(out, points)]

    def _imu_arrays(self, imu_data):
        ts, g = imu_to_arrays(imu_data)
        self._upload_imu(ts, g)
        return ts, g

    # ---- array fast path ------------------------------------------------------------------
    def compensate_arrays(self, xyz, timestamp_ns, frame_start_ns: int, imu_ts, gyro, *,
                          intensity=None) -> np.ndarray:
        """(N,3) points with absolute int64 ns timestamps -> compensated (N,3) float64 (float64
        arithmetic on the given coordinates)."""
        xyz = np.asarray(xyz, dtype=np.float64).reshape(-1, 3)
        if not self.enable_compensation or len(imu_ts) == 0:
            return xyz.copy()
        n = xyz.shape[0]
        if n == 0:
            return np.zeros((0, 3))
        imu_ts = np.ascontiguousarray(imu_ts, dtype=np.int64)
        self._upload_imu(imu_ts, np.ascontiguousarray(gyro, dtype=np.float64).reshape(-1, 3))
        return self._compensate_uploaded(xyz, timestamp_ns, frame_start_ns, intensity)

    def _compensate_uploaded(self, xyz, timestamp_ns, frame_start_ns: int, intensity=None) -> np.ndarray:
        """The device call with the IMU table already on the context (one frame)."""
        n = xyz.shape[0]
        t_rel = np.asarray(timestamp_ns, dtype=np.int64).reshape(-1) - int(frame_start_ns)
        if t_rel.shape != (n,):
            raise ValueError(f"one timestamp per point expected ({n}), got {t_rel.shape}")
        pts = xyz if intensity is None else np.column_stack([xyz, np.asarray(intensity, np.float64)])
        out = deskew_points_f64(self.context, "imu", [n], pts, t_rel, frame_start_ns=[int(frame_start_ns)])
        return out[:, :3]

    # ---- per-frame driver (CSIM:2086-2105), one launch for all frames --------------------------
    def apply_motion_compensation(self, frames_data: List[dict], imu_data: List[IMUData]) -> List[dict]:
        out = []
        if not self.enable_compensation or not imu_data:
            for fr in frames_data:
                c = fr.copy()
                c["motion_compensated"] = True
                out.append(c)
            return out
        self._imu_arrays(imu_data)
        counts = np.array([len(fr["points"]) for fr in frames_data], np.int64)
        pts_all = [p for fr in frames_data for p in fr["points"]]
        if pts_all:
            xyz = np.array([(p.x, p.y, p.z) for p in pts_all], dtype=np.float64).reshape(-1, 3)
            starts = np.array([int(fr["timestamp"]) for fr in frames_data], np.int64)
            t_rel = np.fromiter((p.timestamp for p in pts_all), np.int64, len(pts_all)) - np.repeat(starts, counts)
            res = deskew_points_f64(self.context, "imu", counts, xyz, t_rel, frame_start_ns=starts)
        k = 0
        for fr in frames_data:
            c = fr.copy()
            pts = fr["points"]
            if pts:
                cls = type(pts[0])
                c["points"] = [cls(x=float(res[k + i, 0]), y=float(res[k + i, 1]), z=float(res[k + i, 2]),
                                   intensity=p.intensity, timestamp=p.timestamp, ring=p.ring, tag=p.tag)
                               for i, p in enumerate(pts)]
                k += len(pts)
            else:
                c["points"] = []
            c["motion_compensated"] = True
            out.append(c)
        return out
