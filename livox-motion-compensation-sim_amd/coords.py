"""Drop-in ``CoordinateTransformer`` (CSIM:145-233) and the frame transform of
``LiDARMotionSimulator._transform_coordinates`` (CSIM:2107-2180) — SURVEY §8f row 4.

The 4x4 matrices are built on the host exactly as the reference does (Rz Ry Rx, ``np.linalg.inv``
for the reverse direction); the per-point work ``T @ [p, 1]`` runs on the caller's float64 rows in
libmcdeskew.so (``mc_affine_rows_f64``: numpy's accumulation order, so the outputs equal the
reference's bit for bit), all frames of a run in one launch.  Homogeneous (N,4) input uses its 4th
column as w, like CSIM:226-229.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from .compensator import LiDARPoint
from .runtime import Context, default_context

logger = logging.getLogger(__name__)

try:  # CSIM:47-52: the UTM offset needs the optional `utm` package
    import utm  # type: ignore
    UTM_AVAILABLE = True
except ImportError:
    utm = None
    UTM_AVAILABLE = False


class CoordinateSystem:
    """CSIM:145-151."""
    SENSOR = "sensor"
    VEHICLE = "vehicle"
    LOCAL = "local"
    UTM = "utm"
    WGS84 = "wgs84"


@dataclass
class GPSData:
    """CSIM:108-118."""
    timestamp: int
    latitude: float
    longitude: float
    altitude: float
    velocity_x: float
    velocity_y: float
    velocity_z: float
    heading: float


def _euler_matrix(roll, pitch, yaw) -> np.ndarray:
    cr, sr, cp, sp, cy, sy = np.cos(roll), np.sin(roll), np.cos(pitch), np.sin(pitch), np.cos(yaw), np.sin(yaw)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


class CoordinateTransformer:
    """GPU-backed drop-in for livox_mid70_complete_simulator.CoordinateTransformer."""

    def __init__(self, context: Context | None = None):
        self.transformations: Dict[tuple, np.ndarray] = {}
        self._context = context
        self._setup_default_transformations()

    @property
    def context(self) -> Context:
        if self._context is None:
            self._context = default_context()
        return self._context

    def _setup_default_transformations(self):
        # CSIM:160-174: identities and sensor -> vehicle (1.5 m above ground)
        self.transformations[(CoordinateSystem.SENSOR, CoordinateSystem.SENSOR)] = np.eye(4)
        self.transformations[(CoordinateSystem.VEHICLE, CoordinateSystem.VEHICLE)] = np.eye(4)
        T_sv = np.eye(4)
        T_sv[2, 3] = 1.5
        self.transformations[(CoordinateSystem.SENSOR, CoordinateSystem.VEHICLE)] = T_sv

    def set_transformation(self, from_frame: str, to_frame: str, translation: List[float], rotation: List[float]):
        """CSIM:176-185: the transform and its inverse."""
        T = self._create_transform_matrix(translation, rotation)
        self.transformations[(from_frame, to_frame)] = T
        self.transformations[(to_frame, from_frame)] = np.linalg.inv(T)

    def _create_transform_matrix(self, translation: List[float], rotation: List[float]) -> np.ndarray:
        """CSIM:187-212."""
        roll, pitch, yaw = rotation
        T = np.eye(4)
        T[:3, :3] = _euler_matrix(roll, pitch, yaw)
        T[:3, 3] = translation
        return T

    def transform_points(self, points: np.ndarray, from_frame: str, to_frame: str) -> np.ndarray:
        """CSIM:214-233: (N,3) -> (N,3) float64; (N,4) input is homogeneous as it is; a missing
        transformation logs a warning and returns ``points`` itself."""
        if (from_frame, to_frame) not in self.transformations:
            logger.warning(f"No transformation available from {from_frame} to {to_frame}")
            return points
        return self.transform_frames([points], from_frame, to_frame)[0]

    def transform_frames(self, frames: Sequence[np.ndarray], from_frame: str, to_frame: str) -> List[np.ndarray]:
        """transform_points over many clouds in one launch (all (N_i,3) or all (N_i,4))."""
        T = self.transformations[(from_frame, to_frame)]
        return transform_arrays(frames, T, context=self.context)


def transform_arrays(frames: Sequence[np.ndarray], T, context: Context | None = None,
                     per_point: bool = False) -> List[np.ndarray]:
    """T @ [p, 1] (or T @ p for (N,4) homogeneous rows) for every cloud; one matrix for all, or one
    per cloud ((F,4,4) / (F,3,4)).  Returns (N_i, 3) float64 arrays, computed in float64 on the
    device with numpy's accumulation order: equal to the reference's values bit for bit
    (mc_affine_rows_f64).  Each cloud is one ``T @ points.T`` product; ``per_point`` makes every
    point its own (1, 3) product, as _transform_coordinates' loop does (CSIM:2117-2141) — numpy
    rounds a one-point product differently."""
    arrs = [np.asarray(f) for f in frames]
    if any(a.ndim != 2 for a in arrs):
        raise IndexError("tuple index out of range")     # points.shape[1] on a 1-D array (CSIM:223)
    widths = {a.shape[1] if a.ndim == 2 else -1 for a in arrs}
    if len(widths) > 1 or not widths <= {3, 4}:
        w = next(iter(widths - {3, 4}), None)
        raise ValueError(f"matmul: Input operand 1 has a mismatch in its core dimension 0, with gufunc signature "
                         f"(n?,k),(k,m?)->(n?,m?) (size {w} is different from 4)")
    counts = np.array([len(a) for a in arrs], np.int64)
    if not arrs or counts.sum() == 0:
        return [np.zeros((len(a), 3)) for a in arrs]
    ctx = context or default_context()
    rows = arrs[0] if len(arrs) == 1 else np.concatenate(arrs)
    out = ctx.affine_rows(counts, rows, T, per_row=per_point)
    return [out[o:o + n] for o, n in zip(np.concatenate([[0], np.cumsum(counts)[:-1]]), counts)]


def find_closest_gps_sample(gps_data: List[GPSData], timestamp_ns: int) -> Optional[GPSData]:
    """CSIM:2165-2180: first sample with the smallest |Δt|."""
    if not gps_data:
        return None
    ts = np.array([s.timestamp for s in gps_data], np.int64)
    return gps_data[int(np.argmin(np.abs(ts - int(timestamp_ns))))]


def transform_coordinates(frames_data: List[Dict], target_system: str, gps_data: List[GPSData],
                          transformer: CoordinateTransformer) -> List[Dict]:
    """CSIM:2107-2163 with the per-point loop as one device launch over every frame: UTM targets
    add the closest GPS fix's UTM easting/northing (unchanged without the `utm` package, like the
    reference); other targets apply transformer's sensor -> target matrix (unchanged when missing)."""
    frames_xyz = [np.array([[p.x, p.y, p.z] for p in fr["points"]], np.float64).reshape(-1, 3) for fr in frames_data]
    if target_system == CoordinateSystem.UTM and gps_data:
        # per frame a pure translation by the fix's UTM easting / northing, applied on the device
        Ts = np.tile(np.eye(4), (len(frames_data), 1, 1))
        for f, fr in enumerate(frames_data):
            s = find_closest_gps_sample(gps_data, fr["timestamp"])
            if s is not None and UTM_AVAILABLE:
                try:
                    ux, uy, _, _ = utm.from_latlon(s.latitude, s.longitude)
                    Ts[f, :2, 3] = (ux, uy)
                except Exception:
                    pass
        moved = Ts[:, :2, 3].any(axis=1)
        new_xyz = list(frames_xyz)
        if moved.any():
            # CSIM:2132 point + [utm_x, utm_y, 0]: a plain add per coordinate on the device (no
            # products: a non-finite coordinate stays in its own column, as in the reference)
            sel = np.flatnonzero(moved)
            xs = [frames_xyz[f] for f in sel]
            counts = np.array([len(x) for x in xs], np.int64)
            if counts.sum() > 0:
                ctx = transformer.context or default_context()
                out = ctx.affine_rows(counts, np.concatenate(xs), Ts[sel][:, :3, :4], translate=True)
                for f, o, k in zip(sel, np.concatenate([[0], np.cumsum(counts)[:-1]]), counts):
                    new_xyz[f] = out[o:o + k]
    elif (CoordinateSystem.SENSOR, target_system) in transformer.transformations:
        # CSIM:2137-2139: transform_points on one (1, 3) point at a time
        new_xyz = transform_arrays(frames_xyz, transformer.transformations[(CoordinateSystem.SENSOR, target_system)],
                                   context=transformer.context, per_point=True)
    else:
        logger.warning(f"No transformation available from {CoordinateSystem.SENSOR} to {target_system}")
        new_xyz = frames_xyz
    out = []
    for fr, xyz in zip(frames_data, new_xyz):
        pts = [LiDARPoint(x=float(x), y=float(y), z=float(z), intensity=p.intensity, timestamp=p.timestamp,
                          ring=p.ring, tag=p.tag) for (x, y, z), p in zip(xyz, fr["points"])]
        nf = fr.copy()
        nf["points"] = pts
        nf["coordinate_system"] = target_system
        out.append(nf)
    return out
