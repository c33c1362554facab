"""Drop-in ``LiDARMotionSimulator`` for the reference's alignment path (LMC:274-859).

Same constructor semantics (defaults, validation, merge, global seeding: LMC:275-295), same
pose-table producers (LMC:361-428), and ``transform_pointcloud`` with the reference's exact
signature (LMC:772-776) — but the point work runs in the gfx950 kernels of libmcdeskew.so.
The batched entry points replace the reference's per-frame Python loop (LMC:802-832) with ONE
launch over a ragged batch of frames:

  align_frames(frames, transformations)      explicit pose per frame      (MC_POSE_DIRECT)
  run_alignment(scans, trajectory, times)     LMC:804-831 pose selection  (MC_POSE_SEARCHSORTED)
  deskew_frames(frames, t_ns, ...)            per-point SLERP/LERP pose   (build-added mode)
  merge_aligned(aligned)                      LMC:887-889 np.vstack

Around the path, also on the GPU: scan_environment / scan_frames / simulate_frames / run_simulation
(LMC:701-858, the scan feeding the alignment without leaving HBM) and the byte-exact writers
save_pcd / save_lvx / save_results (LMC:860-990; CSVs through pandas, LAS through laspy when it is
installed, as in the reference).  Scene synthesis, plots and reports (LMC:430-699, 992-1173) are
not provided.
"""
from __future__ import annotations

import os
from ctypes import c_double, c_int64
from typing import Dict, List, Optional

import numpy as np

from . import _lib
from . import codecs as _codecs
from . import config as _config
from . import trajectory as _traj
from ._lib import check, fptr, ptr
from .runtime import Context, default_context, deskew_points_f64, host_pool

POOLED_ROWS = 1 << 20   # results of at least this many rows (32 MB) come from the recycled host blocks


class LiDARMotionSimulator:
    """GPU-backed drop-in for lidar_motion_compensation.LiDARMotionSimulator's alignment path."""

    def __init__(self, config: Optional[Dict] = None, *, context: Context | None = None):
        # LMC:282-288: defaults, validate the override, merge, seed the global RNG
        self.config = self.default_config()
        if config:
            self._validate_config(config)
            self.config.update(config)
        np.random.seed(self.config["random_seed"])
        self._performance_stats = {"scan_times": [], "transform_times": [], "total_points_processed": 0}
        self._context = context

    # ---- config contract (LMC:297-359) ---------------------------------------------------
    def default_config(self):
        return _config.default_config()

    def _validate_config(self, config: Dict) -> None:
        _config.validate_config(config)

    # ---- pose tables (LMC:361-428, 792-793) ----------------------------------------------
    def generate_trajectory(self):
        return _traj.generate_trajectory(self.config)

    def add_sensor_noise(self, trajectory):
        return _traj.add_sensor_noise(trajectory, self.config)

    def lidar_times(self) -> np.ndarray:
        return _traj.lidar_times(self.config)

    # ---- device plumbing -------------------------------------------------------------------
    @property
    def context(self) -> Context:
        if self._context is None:
            self._context = default_context()
        return self._context

    @staticmethod
    def _check_points(points):
        points = np.asarray(points)
        if points.ndim != 2:
            raise IndexError(f"too many indices for array: array is {points.ndim}-dimensional, but 2 were indexed")
        if points.shape[1] < 4:
            raise IndexError(f"index 3 is out of bounds for axis 1 with size {points.shape[1]}")
        return points

    # ---- the hot path ---------------------------------------------------------------------
    def transform_pointcloud(self, points, transformation):
        """LMC:772-776: p' = R_xyz(rotation) p + translation, intensity passed through.

        points (N, >=4) -> new (N, 4) float64 array; input untouched; (0,4) -> (0,4).
        """
        points = self._check_points(points)
        rot = np.ascontiguousarray(transformation["rotation"], dtype=np.float64).reshape(3)
        trans = np.ascontiguousarray(transformation["translation"], dtype=np.float64).reshape(3)
        if points.shape[0] == 0:
            return np.zeros((0, 4))
        # one frame per call (the reference's loop): the float64 kernel on pinned host memory
        p = np.ascontiguousarray(points, dtype=np.float64)
        out = np.empty((p.shape[0], 4))
        ctx = self.context
        rc = ctx.lib.mc_transform_pointcloud_f64(ctx.handle, fptr(p, c_double), p.shape[0], p.shape[1],
                                                 fptr(rot, c_double), fptr(trans, c_double), fptr(out, c_double))
        if rc:
            check(rc, "transform_pointcloud")
        return out

    def align_frames(self, frames: List[np.ndarray], transformations: List[dict]) -> List[np.ndarray]:
        """Batched transform_pointcloud: frame i uses transformations[i]; one kernel launch."""
        if len(frames) != len(transformations):
            raise ValueError("one transformation per frame expected")
        frames = [self._check_points(f) for f in frames]
        if not frames:
            return []
        rot = np.stack([np.asarray(t["rotation"], np.float64).reshape(3) for t in transformations])
        trans = np.stack([np.asarray(t["translation"], np.float64).reshape(3) for t in transformations])
        if sum(f.shape[0] for f in frames) == 0:
            return [np.zeros((0, 4)) for _ in frames]
        self.context.set_trajectory(np.arange(len(frames), dtype=np.float64), trans, rot)
        return self._align_host(frames, None, _lib.MC_POSE_DIRECT)

    def _align_host(self, frames, times, pose_select) -> List[np.ndarray]:
        """Host arrays in, host arrays out: one float64 launch over all frames on pinned,
        device-mapped memory (mc_align_frames_host_f64); poses from the uploaded trajectory."""
        ctx = self.context
        src = [f if f.dtype == np.float64 and f.flags.c_contiguous else np.ascontiguousarray(f, dtype=np.float64)
               for f in frames]
        F = len(src)
        counts = np.fromiter((f.shape[0] for f in src), np.int64, F)
        lds = np.fromiter((f.shape[1] for f in src), np.int64, F)
        offs = np.concatenate([[0], np.cumsum(counts)])
        n = int(offs[-1])
        # one allocation, frames are views; a large result takes a recycled block when one is idle
        # (no first-touch page faults), runtime.HostPool
        out = host_pool().empty((n, 4)) if n >= POOLED_ROWS else np.empty((n, 4))
        fp = np.fromiter((f.__array_interface__["data"][0] for f in src), np.uintp, F)
        op = (out.__array_interface__["data"][0] + 32 * offs[:-1]).astype(np.uintp)
        t = None if times is None else np.ascontiguousarray(times, dtype=np.float64)
        check(ctx.lib.mc_align_frames_host_f64(ctx.handle, F, fp.ctypes.data, ptr(counts, c_int64),
                                               ptr(lds, c_int64), ptr(t, c_double), pose_select, op.ctypes.data),
              "align_frames")
        return [out[offs[f]:offs[f + 1]] for f in range(F)]

    def run_alignment(self, scans: List[np.ndarray], trajectory: dict,
                      times: Optional[np.ndarray] = None) -> List[np.ndarray]:
        """The reference's frame loop (LMC:802-832) for given local scans: per frame the
        'next-or-equal' pose (searchsorted + clamp, LMC:804-806) of position_gps /
        orientation_imu, then transform_pointcloud — all frames in one launch."""
        if times is None:
            times = self.lidar_times()[: len(scans)]
        times = np.asarray(times, dtype=np.float64)
        if len(times) != len(scans):
            raise ValueError("one frame time per scan expected")
        scans = [self._check_points(s) for s in scans]
        if not scans or sum(s.shape[0] for s in scans) == 0:
            return [np.zeros((0, 4)) for _ in scans]
        self.context.set_trajectory(trajectory["time"], trajectory["position_gps"], trajectory["orientation_imu"])
        return self._align_host(scans, times, _lib.MC_POSE_SEARCHSORTED)

    def deskew_frames(self, frames: List[np.ndarray], t_ns: List[np.ndarray], trajectory: dict,
                      times: Optional[np.ndarray] = None) -> List[np.ndarray]:
        """Per-point motion compensation into the global frame: every return at time
        t_frame + t_ns*1e-9 gets the SLERP/LERP-interpolated pose of the trajectory
        (position_gps, orientation_imu), p' = R(q(t)) p + pos(t).  Computed in float64 on the given
        float64 rows, one launch for all frames (mc_deskew_points_f64); device-resident frames take
        ``Context.deskew(mode="pose_slerp")`` instead."""
        if times is None:
            times = self.lidar_times()[: len(frames)]
        times = np.asarray(times, dtype=np.float64)
        if not (len(times) == len(frames) == len(t_ns)):
            raise ValueError("frames, t_ns and times must have the same length")
        frames = [self._check_points(f) for f in frames]
        counts = np.array([f.shape[0] for f in frames], np.int64)
        for f, t in zip(frames, t_ns):
            if np.shape(t) != (f.shape[0],):
                raise ValueError("one timestamp per point expected")
        if not frames or counts.sum() == 0:
            return [np.zeros((0, 4)) for _ in frames]
        ctx = self.context
        ctx.set_trajectory(trajectory["time"], trajectory["position_gps"], trajectory["orientation_imu"])
        out = deskew_points_f64(ctx, "pose_slerp", counts, _stack_aos(frames),
                                np.concatenate([np.asarray(t, np.int64) for t in t_ns]), frame_times=times)
        offs = np.concatenate([[0], np.cumsum(counts)])
        return [out[offs[f]:offs[f + 1]] for f in range(len(frames))]

    # ---- scanning (LMC:701-770) and the frame loop (LMC:778-858) ----------------------------
    def _load_environment(self, environment) -> np.ndarray:
        """Make ``environment`` the context's scene.  The context compares the scene's bytes with
        the one it holds and uploads only on a difference, so simulators sharing a context, and
        in-place edits of one array, always scan the scene they pass."""
        env = np.asarray(environment)
        self.context.set_environment(env)
        return env

    def scan_environment(self, environment, sensor_pose):
        """LMC:701-770: the sensor-frame scan of ``environment`` from one pose (``position`` and
        ``orientation`` rad), (n, 4) [x, y, z, intensity]; draws the range noise from the global
        RNG like the reference."""
        self._load_environment(environment)
        ctx = self.context
        ctx.set_trajectory([0.0], np.asarray(sensor_pose["position"], np.float64).reshape(1, 3),
                           np.asarray(sensor_pose["orientation"], np.float64).reshape(1, 3))
        _, local, _ = ctx.scan_rows([0.0], self.config, pose_select="direct", aligned=False)
        return local

    def scan_frames(self, environment, trajectory: dict, times: Optional[np.ndarray] = None):
        """Every frame's scan (LMC:802-817 pose selection + 815 scan) as one device batch of float32
        columns (the hot path's input layout), noise drawn in frame order from the global RNG.
        Returns the device ``Batch`` of local scans."""
        if times is None:
            times = self.lidar_times()
        self._load_environment(environment)
        ctx = self.context
        ctx.set_trajectory(trajectory["time"], trajectory["position_gps"], trajectory["orientation_imu"])
        return ctx.scan(np.asarray(times, np.float64), self.config, pose_select="searchsorted")

    def simulate_frames(self, environment, trajectory: dict, times: Optional[np.ndarray] = None) -> dict:
        """The frame loop of run_simulation (LMC:802-850) with both point stages on the GPU in one
        pass: every frame's scan (LMC:815) and its alignment with the same pose (LMC:826-831) are
        written by one kernel as the reference's float64 arrays, bit-identical to the reference's
        values (mc_scan_emit_f64).  Returns run_simulation's dict (LMC:852-858)."""
        if times is None:
            times = self.lidar_times()
        times = np.asarray(times, np.float64)
        self._load_environment(environment)
        ctx = self.context
        ctx.set_trajectory(trajectory["time"], trajectory["position_gps"], trajectory["orientation_imu"])
        self._drop_rows()
        counts, local, aligned, (d_local, d_aligned) = ctx.scan_rows(times, self.config, pose_select="searchsorted",
                                                                       keep_device=True)
        offs = np.concatenate([[0], np.cumsum(counts)])
        idx = np.clip(np.searchsorted(trajectory["time"], times), 0, len(trajectory["time"]) - 1)
        raw, al, motion = [], [], []
        for i, (t, k) in enumerate(zip(times, idx)):
            pose = {"position": trajectory["position_gps"][k], "orientation": trajectory["orientation_imu"][k],
                    "velocity": trajectory["velocity"][k]}
            raw.append({"frame_id": i, "timestamp": t, "points_local": local[offs[i]:offs[i + 1]], "sensor_pose": pose})
            al.append(aligned[offs[i]:offs[i + 1]])
            p, o, v = pose["position"], pose["orientation"], pose["velocity"]
            motion.append({"frame_id": i, "timestamp": t,
                           "gps_lat": p[1] / 111320.0 + 40.0,
                           "gps_lon": p[0] / (111320.0 * np.cos(np.radians(40.0))) - 74.0,
                           "gps_alt": p[2], "imu_roll": o[0], "imu_pitch": o[1], "imu_yaw": o[2],
                           "vel_x": v[0], "vel_y": v[1], "vel_z": v[2]})
        if d_local is not None:
            self._rows = _DeviceRows(counts, local, aligned, d_local, d_aligned, raw, al)
        return {"raw_scans": raw, "aligned_pointclouds": al, "motion_data": motion,
                "trajectory": trajectory, "environment": environment}

    def _drop_rows(self):
        rows, self._rows = getattr(self, "_rows", None), None
        if rows is not None:
            rows.close()

    def _rows_of(self, results) -> Optional["_DeviceRows"]:
        rows = getattr(self, "_rows", None)
        return rows if rows is not None and rows.matches(results) else None

    def run_simulation(self, environment):
        """LMC:778-858 given the scene: trajectory + sensor noise (LMC:784-785, global RNG), then
        simulate_frames over the lidar time grid.  Scene synthesis (LMC:430-699) is not provided
        (DESIGN.md §1): pass the environment array."""
        trajectory = self.add_sensor_noise(self.generate_trajectory())
        return self.simulate_frames(environment, trajectory, self.lidar_times())

    # ---- file output (LMC:932-948, 965-990) ----------------------------------------------------
    def save_pcd(self, points, filename):
        """LMC:932-948: ASCII PCD v0.7, lines formatted on the GPU (byte-identical)."""
        _codecs.save_pcd(points, filename, self.context)

    def save_las(self, points, filename):
        """LMC:950-963 through laspy (a host file format; raises ImportError without laspy)."""
        import laspy   # noqa: F401  (optional dependency, as in the reference)
        header = laspy.LasHeader(point_format=3, version="1.2")
        las = laspy.LasData(header)
        las.x, las.y, las.z = points[:, 0], points[:, 1], points[:, 2]
        las.intensity = (points[:, 3] * 65535).astype(np.uint16)
        las.write(filename)

    def save_results(self, results, output_dir="lidar_simulation_output"):
        """LMC:860-931: motion / trajectory CSVs, per-frame raw and aligned PCDs, the merged PCDs,
        LAS and LVX.  Every PCD's point lines come from one GPU launch pair over all frames; the
        merged files reuse the frames' lines (a vstack of the clouds prints the same lines)."""
        import pandas as pd
        os.makedirs(output_dir, exist_ok=True)
        print(f"Saving results to {output_dir}...")
        pd.DataFrame(results["motion_data"]).to_csv(os.path.join(output_dir, "motion_data.csv"), index=False)
        raw = [s["points_local"] for s in results["raw_scans"]]
        aligned = list(results["aligned_pointclouds"])
        rows = self._rows_of(results)
        if rows is not None:     # simulate_frames' own result: its rows are still on the device
            raw_b = _codecs.encode_pcd_bodies_device_rows(rows.d_local, rows.counts)
            al_b = _codecs.encode_pcd_bodies_device_rows(rows.d_aligned, rows.counts)
        else:
            bodies = _codecs.encode_pcd_bodies(raw + aligned, self.context) if raw or aligned else []
            raw_b, al_b = bodies[:len(raw)], bodies[len(raw):]
        pcd_dir = os.path.join(output_dir, "raw_scans_pcd")
        os.makedirs(pcd_dir, exist_ok=True)
        for s, pts, body in zip(results["raw_scans"], raw, raw_b):
            _write(os.path.join(pcd_dir, f'frame_{s["frame_id"]:04d}.pcd'), _codecs.pcd_header(len(pts)) + body)
        aligned_dir = os.path.join(output_dir, "aligned_scans_pcd")
        os.makedirs(aligned_dir, exist_ok=True)
        for i, (pts, body) in enumerate(zip(aligned, al_b)):
            _write(os.path.join(aligned_dir, f"aligned_frame_{i:04d}.pcd"), _codecs.pcd_header(len(pts)) + body)
        merged_aligned = None
        if aligned and all(len(pc) > 0 for pc in aligned):      # LMC:887
            n = sum(len(pc) for pc in aligned)
            _write(os.path.join(output_dir, "merged_aligned.pcd"), _codecs.pcd_header(n) + b"".join(al_b))
            merged_aligned = self.merge_aligned(aligned)
        else:
            print("Warning: No aligned point clouds to merge")
        keep = [i for i, pts in enumerate(raw) if len(pts) > 0]
        if keep:
            n = sum(len(raw[i]) for i in keep)
            _write(os.path.join(output_dir, "merged_raw_overlapped.pcd"),
                   _codecs.pcd_header(n) + b"".join(raw_b[i] for i in keep))
        else:
            print("Warning: No raw point clouds to merge")
        try:
            if merged_aligned is None:
                # LMC:903 reads merged_aligned, unbound when LMC:887 skipped the merge
                raise UnboundLocalError("local variable 'merged_aligned' referenced before assignment")
            self.save_las(merged_aligned, os.path.join(output_dir, "merged_aligned.las"))
            print("LAS format saved successfully")
        except Exception as e:
            print(f"Could not save LAS format: {e}")
        try:
            self.save_lvx(results, os.path.join(output_dir, "lidar_data"))
            print("LVX formats saved successfully")
        except Exception as e:
            print(f"Could not save LVX formats: {e}")
        tr = results["trajectory"]
        pd.DataFrame({"time": tr["time"], "x": tr["position"][:, 0], "y": tr["position"][:, 1],
                      "z": tr["position"][:, 2], "x_gps": tr["position_gps"][:, 0], "y_gps": tr["position_gps"][:, 1],
                      "z_gps": tr["position_gps"][:, 2]}).to_csv(os.path.join(output_dir, "trajectory.csv"), index=False)
        print("Results saved successfully!")
        return output_dir

    def save_lvx(self, results, base_filename):
        """LMC:965-990: the raw (local) scans of ``results`` as ``<base_filename>.lvx``."""
        frames_data = [{"frame_id": s["frame_id"], "timestamp": s["timestamp"], "points": s["points_local"]}
                       for s in results["raw_scans"]]
        print("Generating corrected LVX format...")
        rows = self._rows_of(results)
        try:
            w = _codecs.LivoxLVXWriter(self.context)
            if rows is not None:   # simulate_frames' own result: encode from its device rows
                w._write(f"{base_filename}.lvx", frames_data,
                         lambda: _codecs.encode_lvx_device_rows(rows.d_local, rows.counts, frames_data))
            else:
                w.write_compatible_lvx(f"{base_filename}.lvx", frames_data)
            print(f"✅ Corrected LVX format: {base_filename}.lvx")
        except Exception as e:
            print(f"❌ LVX generation failed: {e}")
        print(f"Processed {len(frames_data)} frames with corrected LVX implementation")

    @staticmethod
    def merge_aligned(aligned: List[np.ndarray]) -> np.ndarray:
        """LMC:887-889: frame-ordered concatenation of the aligned clouds."""
        if not aligned:
            return np.zeros((0, 4))
        return np.vstack(aligned)


def _digest(a: np.ndarray) -> int:
    import xxhash
    return xxhash.xxh3_64_intdigest(memoryview(np.ascontiguousarray(a)).cast("B"))


class _DeviceRows:
    """The device copies of one simulate_frames result's local and aligned rows (mc_scan_emit_f64's
    (N, 4) float64 output), so save_results / save_lvx encode them without staging and uploading the
    host arrays again.  Used only while the result still holds the very lists and arrays
    simulate_frames returned and their bytes are unchanged (identity + a 64-bit xxh3 digest of each
    row array): any replaced frame or in-place edit sends the writers back to the host arrays."""

    def __init__(self, counts, local, aligned, d_local, d_aligned, raw_list, al_list):
        self.counts = np.ascontiguousarray(counts, np.int64)
        self.local, self.aligned = local, aligned
        self.d_local, self.d_aligned = d_local, d_aligned
        self.raw_list, self.al_list = raw_list, al_list
        self.local_views = [s["points_local"] for s in raw_list]
        self.al_views = list(al_list)
        try:
            self.h = (_digest(local), _digest(aligned))
        except ImportError:
            self.h = None

    def matches(self, results) -> bool:
        if self.h is None or self.d_aligned is None:
            return False
        raw, al = results.get("raw_scans"), results.get("aligned_pointclouds")
        if raw is not self.raw_list or al is not self.al_list or len(raw) != len(self.local_views) \
                or len(al) != len(self.al_views):
            return False
        if any(s.get("points_local") is not v for s, v in zip(raw, self.local_views)):
            return False
        if any(a is not v for a, v in zip(al, self.al_views)):
            return False
        return (_digest(self.local), _digest(self.aligned)) == self.h

    def close(self):
        for b in (self.d_local, self.d_aligned):
            if b is not None:
                b.close()


def _stack_aos(frames: List[np.ndarray]) -> np.ndarray:
    """Frame-ordered (N, ld) float64 stack; ld = the narrowest frame width (>= 4)."""
    ld = min(f.shape[1] for f in frames)
    if len(frames) == 1:
        return np.ascontiguousarray(frames[0][:, :ld], dtype=np.float64)
    return np.ascontiguousarray(np.concatenate([f[:, :ld] for f in frames]), dtype=np.float64)


def _write(path: str, data: bytes) -> None:
    with open(path, "wb") as f:
        f.write(data)
