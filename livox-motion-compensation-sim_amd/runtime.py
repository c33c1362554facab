"""Device context and blocked-CSR frame batches — thin Python objects over the C-ABI handles.

A ``Context`` is one HIP device + stream (one per process/rank, like the C-ABI's mc_ctx).  A
``Batch`` is a device-resident ragged batch of frames laid out as float32 columns
x|y|z|intensity (+ int32 t_ns) in HBM; it is what one launch of the hot kernel consumes
(DESIGN.md §3).
"""
from __future__ import annotations

import ctypes
import os
import weakref
from ctypes import c_double, c_float, c_int, c_int32, c_int64, c_void_p

import numpy as np

from . import _lib
from ._lib import check, ptr


def _f64(a, shape_tail=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape_tail is not None and a.shape[1:] != shape_tail:
        raise ValueError(f"expected shape (n,{','.join(map(str, shape_tail))}), got {a.shape}")
    return a


class Context:
    """One device + stream.  ``device`` defaults to $MCDESKEW_DEVICE, else $LOCAL_RANK modulo the
    visible devices (a launcher that gives each rank its own HIP_VISIBLE_DEVICES leaves every rank
    one device, 0), else 0.  ``lib_path`` loads an alternative build of the library (A/B variant runs
    in one process)."""

    def __init__(self, device: int | None = None, lib_path: str | None = None):
        self.lib = _lib.load(lib_path) if lib_path else _lib.load()
        if device is None and "MCDESKEW_DEVICE" in os.environ:
            device = int(os.environ["MCDESKEW_DEVICE"])
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
            n = c_int(0)
            if device > 0 and self.lib.mc_device_count(ctypes.byref(n)) == 0 and n.value > 0:
                device %= n.value
        h = c_void_p()
        check(self.lib.mc_create(int(device), ctypes.byref(h)), "mc_create")
        self.handle = h
        self.device = device
        self._fin = weakref.finalize(self, self.lib.mc_destroy, h)

    @staticmethod
    def device_count() -> int:
        lib = _lib.load()
        n = c_int(0)
        check(lib.mc_device_count(ctypes.byref(n)), "mc_device_count")
        return n.value

    def pci_bus_id(self) -> str:
        buf = (ctypes.c_char * 64)()
        check(self.lib.mc_device_pci_bus_id(int(self.device), buf, 64), "pci_bus_id")
        return buf.value.decode()

    def close(self):
        self._fin()

    def sync(self):
        check(self.lib.mc_sync(self.handle), "mc_sync")

    # ---- pose sources -------------------------------------------------------------------
    def set_trajectory(self, time, position, rpy):
        """Pose table (LMC:361-428): time (T,), position_gps (T,3), orientation_imu (T,3) rad."""
        t = _f64(np.atleast_1d(time))
        p = _f64(np.atleast_2d(position), (3,))
        r = _f64(np.atleast_2d(rpy), (3,))
        if not (len(t) == len(p) == len(r)):
            raise ValueError("time / position / rpy lengths differ")
        check(self.lib.mc_set_trajectory(self.handle, len(t), ptr(t, c_double), ptr(p, c_double),
                                         ptr(r, c_double)), "set_trajectory")

    def set_imu(self, timestamp_ns, gyro):
        """IMU samples (CSIM:98-106): int64 ns timestamps (sorted), gyro (M,3) rad/s."""
        ts = np.ascontiguousarray(timestamp_ns, dtype=np.int64)
        g = _f64(np.atleast_2d(gyro), (3,))
        if len(ts) != len(g):
            raise ValueError("timestamp / gyro lengths differ")
        last = getattr(self, "_imu_last", None)
        if (last is not None and last[1].shape == g.shape and np.array_equal(last[0], ts)
                and np.array_equal(last[1].view(np.uint64), g.view(np.uint64))):
            return  # the device already holds these exact bytes (-0.0 and NaN payloads included)
        self._imu_last = None
        check(self.lib.mc_set_imu(self.handle, len(ts), ptr(ts, c_int64), ptr(g, c_double)), "set_imu")
        self._imu_last = (ts.copy(), g.copy())

    # ---- batches -------------------------------------------------------------------------
    def batch(self, counts, with_time: bool = False, with_pcd_len: bool = False) -> "Batch":
        return Batch(self, counts, with_time, with_pcd_len)

    def deskew(self, inp: "Batch", out: "Batch | None" = None, mode: str = "frame",
               pose_select: str = "searchsorted") -> "Batch":
        """Launch the hot path on the context stream (asynchronous); returns ``out``."""
        if out is None:
            out = Batch(self, inp.counts, with_time=inp.with_time)
        check(self.lib.mc_deskew(self.handle, inp.handle, out.handle, _lib.MODES[mode],
                                 _lib.POSE_SELECT[pose_select]), f"deskew[{mode}]")
        return out

    def deskew_steps(self, inp: "Batch", out: "Batch", n_steps: int, mode: str = "frame",
                     pose_select: str = "searchsorted", sample_every: int = 0) -> "Batch":
        """``n_steps`` calls of :meth:`deskew` (asynchronous) as n + 1 launches: each step's launch
        also runs the next step's prep (mc_deskew_steps).  ``sample_every``: timing events around
        every n-th step's kernels (:meth:`read_timing`)."""
        check(self.lib.mc_deskew_steps(self.handle, inp.handle, out.handle, _lib.MODES[mode],
                                       _lib.POSE_SELECT[pose_select], int(n_steps), int(sample_every)),
              f"deskew_steps[{mode}]")
        return out

    def tune_order(self, inp: "Batch", out: "Batch", mode: str = "frame", pose_select: str = "searchsorted",
                   launches: int = 8, rounds: int = 4) -> dict:
        """Measure which sub-tile order (dealt / XCD-contiguous) runs ``mode``'s kernel faster on this
        device for batches shaped like ``inp`` and keep it for later launches (mc_tune_order; the
        output does not depend on the order).  Returns {"dealt_us", "xcd_us", "chosen"}."""
        us = np.zeros(2, np.float64)
        ch = c_int32(-1)
        check(self.lib.mc_tune_order(self.handle, inp.handle, out.handle, _lib.MODES[mode], _lib.POSE_SELECT[pose_select],
                                     int(launches), int(rounds), ptr(us, c_double), ctypes.byref(ch)),
              f"tune_order[{mode}]")
        return {"dealt_us": float(us[0]), "xcd_us": float(us[1]),
                "chosen": {0: "dealt", 1: "xcd"}.get(ch.value, None)}

    def transform_affine(self, inp: "Batch", out: "Batch | None" = None, mats=None, w_column: bool = False) -> "Batch":
        """p' = A p + b (CSIM:214-233) with one 3x4 [A | b] for all frames or one per frame;
        ``w_column``: the 4th column is the homogeneous w (p' = A p + b w).  Synchronous."""
        m = np.ascontiguousarray(mats, dtype=np.float64)
        if m.ndim == 2:
            m = m[None]
        if m.shape[1:] not in ((3, 4), (4, 4)):
            raise ValueError(f"expected (3,4) / (4,4) matrices, got {np.shape(mats)}")
        m = np.ascontiguousarray(m[:, :3, :4])
        if out is None:
            out = Batch(self, inp.counts, with_time=False)
        check(self.lib.mc_transform_affine(self.handle, inp.handle, out.handle, len(m), ptr(m, c_double),
                                           int(bool(w_column))), "transform_affine")
        return out

    # ---- scan_environment (LMC:701-770) ----------------------------------------------------
    def set_environment(self, environment):
        """Static scene (E, >=4) float64 [x, y, z, intensity] (LMC:430-699's output), to HBM."""
        env = np.asarray(environment)
        if env.ndim != 2:
            raise IndexError(f"too many indices for array: array is {env.ndim}-dimensional, but 2 were indexed")
        if env.shape[1] < 4:
            raise IndexError(f"index 3 is out of bounds for axis 1 with size {env.shape[1]}")
        # the device holds x, y, z, intensity only: skip the upload when those are the same bytes as
        # the scene already there (whoever uploaded it; compared by value, like set_imu)
        env4 = np.ascontiguousarray(env[:, :4], dtype=np.float64)
        last = getattr(self, "_env_last", None)
        if last is not None and last.shape == env4.shape and np.array_equal(
                last.view(np.uint64), env4.view(np.uint64)):
            return
        self._env_last = None
        check(self.lib.mc_set_environment(self.handle, env4.shape[0], ptr(env4, c_double), 4), "set_environment")
        self._env_last = env4.copy()   # env4 may be a view of the caller's array

    def _scan_count(self, frame_times, config: dict, pose_select: str, rng):
        t = np.ascontiguousarray(np.atleast_1d(frame_times), dtype=np.float64)
        F = len(t)
        par = np.array([config["range_min"], config["range_max"], config["fov_horizontal"],
                        config["fov_vertical"]], np.float64)
        counts = np.zeros(F, np.int64)
        check(self.lib.mc_scan_count(self.handle, F, ptr(t, c_double), _lib.POSE_SELECT[pose_select],
                                     ptr(par, c_double), int(config["points_per_frame"]), ptr(counts, c_int64)),
              "scan_count")
        noise = None
        std = config["lidar_range_noise"]
        if std > 0 and counts.sum() > 0:
            # one draw of sum(n_f) x 3 consumes the legacy normal stream exactly like F per-frame
            # draws of n_f x 3 (frames with no visible point draw nothing in the reference either)
            noise = np.ascontiguousarray(rng.normal(0, std, (int(counts.sum()), 3)), dtype=np.float64)
        return counts, noise

    def scan(self, frame_times, config: dict, pose_select: str = "searchsorted", rng=np.random,
             out: "Batch | None" = None) -> "Batch":
        """All frames' local scans of the scene (LMC:701-770 once per frame of LMC:802-831) in two
        launches into a float32 batch: visibility counts per (frame, scene tile), then in-order
        compaction, the systematic subsample and the range noise.  The trajectory must be set (pose
        per frame as in ``deskew(mode='frame')``).  The noise is drawn here from ``rng`` (numpy's
        global RNG by default) in frame order, exactly as the reference's per-frame
        ``np.random.normal`` calls consume it (LMC:765-768), so seeded runs reproduce its scans."""
        counts, noise = self._scan_count(frame_times, config, pose_select, rng)
        if out is None or not np.array_equal(out.counts, counts):
            out = Batch(self, counts)
        check(self.lib.mc_scan_emit(self.handle, out.handle, ptr(noise, c_double)), "scan_emit")
        return out

    def scan_rows(self, frame_times, config: dict, pose_select: str = "searchsorted", rng=np.random,
                  aligned: bool = True, keep_device: bool = False):
        """:meth:`scan` into the reference's own float64 arrays (mc_scan_emit_f64): returns
        (counts, local, aligned) with local / aligned (N, 4) float64 host arrays, frames back to back
        — scan_environment's output and transform_pointcloud of it with the frame's pose (LMC:815,
        831), equal to the reference's values bit for bit; ``aligned=False``: local only (None).
        ``keep_device``: also return the two device (N, 4) float64 buffers (DeviceBuffer, the
        caller closes them), e.g. for the writers that follow (save_results)."""
        counts, noise = self._scan_count(frame_times, config, pose_select, rng)
        n = int(counts.sum())
        if n == 0:
            empty = (counts, np.zeros((0, 4)), (np.zeros((0, 4)) if aligned else None))
            return empty + ((None, None),) if keep_device else empty
        loc = DeviceBuffer(self, n * 32)
        al = DeviceBuffer(self, n * 32) if aligned else None
        keep = False
        try:
            check(self.lib.mc_scan_emit_f64(self.handle, ptr(noise, c_double), loc.ptr, al.ptr if al else None),
                  "scan_emit_f64")
            host = (counts, loc.to_host(np.float64, (n, 4)), (al.to_host(np.float64, (n, 4)) if al else None))
            keep = keep_device
            return host + ((loc, al),) if keep_device else host
        finally:
            if not keep:
                loc.close()
                if al:
                    al.close()

    def affine_rows(self, counts, rows, mats, per_row: bool = False, translate: bool = False) -> np.ndarray:
        """(T @ [p, w].T).T[:, :3] on float64 rows (mc_affine_rows_f64): rows (N, 3) (w = 1) or
        (N, 4) homogeneous, frames of ``counts`` rows back to back, each frame one numpy product (or,
        with ``per_row``, every row its own one-point product); one (3|4, 4) matrix or one per
        frame.  Returns (N, 3) float64, bit-identical to numpy's (CSIM:230).  ``translate``: the
        rows' x, y, z plus the matrices' translation column only (CSIM:2132's UTM offset add)."""
        c = np.ascontiguousarray(np.atleast_1d(counts), dtype=np.int64)
        r = np.ascontiguousarray(rows, dtype=np.float64)
        m = np.ascontiguousarray(mats, dtype=np.float64)
        if m.ndim == 2:
            m = m[None]
        if m.shape[1:] not in ((3, 4), (4, 4)):
            raise ValueError(f"expected (3,4) / (4,4) matrices, got {np.shape(mats)}")
        m = np.ascontiguousarray(m[:, :3, :4])
        out = np.empty((r.shape[0], 3), np.float64)
        check(self.lib.mc_affine_rows_f64(self.handle, len(c), ptr(c, c_int64), ptr(r, c_double), r.shape[1],
                                          len(m), ptr(m, c_double), 2 if translate else int(bool(per_row)), ptr(out, c_double)),
              "affine_rows")
        return out

    def set_max_grid(self, max_grid: int):
        check(self.lib.mc_set_launch(self.handle, int(max_grid)), "set_launch")

    def timing(self, enable: bool = True):
        check(self.lib.mc_timing_enable(self.handle, int(bool(enable))), "timing_enable")

    def read_timing(self) -> dict:
        mm, pm, lm = c_double(), c_double(), c_double()
        mn, pn, ln = c_int64(), c_int64(), c_int64()
        check(self.lib.mc_timing_read(self.handle, ctypes.byref(mm), ctypes.byref(mn), ctypes.byref(pm),
                                      ctypes.byref(pn)), "timing_read")
        check(self.lib.mc_timing_read_layout(self.handle, ctypes.byref(lm), ctypes.byref(ln)), "timing_read_layout")
        sm, sn, cm, cn = c_double(), c_int64(), c_double(), c_int64()
        check(self.lib.mc_timing_read_scan(self.handle, ctypes.byref(sm), ctypes.byref(sn)), "timing_read_scan")
        check(self.lib.mc_timing_read_codec(self.handle, ctypes.byref(cm), ctypes.byref(cn)), "timing_read_codec")
        return {"main_ms": mm.value, "main_launches": mn.value, "prep_ms": pm.value, "prep_launches": pn.value,
                "layout_ms": lm.value, "layout_launches": ln.value, "scan_ms": sm.value, "scan_launches": sn.value,
                "codec_ms": cm.value, "codec_launches": cn.value}

    def read_timing_each(self, cap: int = 4096) -> list:
        """The main kernels' event times (ms) one by one, in launch order (released; the other timing
        events stay pending for read_timing)."""
        buf = np.zeros(cap, np.float64)
        n = c_int64()
        check(self.lib.mc_timing_read_each(self.handle, ptr(buf, c_double), cap, ctypes.byref(n)), "timing_read_each")
        return buf[:min(n.value, cap)].tolist()

    def read_timing_spans(self, cap: int = 4096) -> list:
        """The timed deskew launches' own execution spans (us): first workgroup start to last
        workgroup end on the device wall clock, in launch order (released)."""
        buf = np.zeros(cap, np.float64)
        n = c_int64()
        check(self.lib.mc_timing_read_spans(self.handle, ptr(buf, c_double), cap, ctypes.byref(n)), "timing_read_spans")
        return buf[:min(n.value, cap)].tolist()

    def device_buffer(self, nbytes: int) -> "DeviceBuffer":
        return DeviceBuffer(self, nbytes)


class HostPool:
    """Recycled host blocks for large host-array results (run_alignment / align_frames): a fresh
    (n, 4) float64 result costs its first-touch page faults (~90 ms for 1.9 GB, as much as moving it
    over PCIe); a block whose previous array has died is handed out again already faulted.  The
    returned array is an ordinary writeable numpy array; its block returns here when the last view of
    it dies and serves the next result it fits (at most twice its size).  At most ``cap`` bytes wait."""

    def __init__(self, cap: int = 8 << 30):
        import threading
        self.cap = int(cap)
        self._free: list = []        # idle blocks (uint8 ndarrays)
        self._busy: dict = {}        # id(proxy) -> block, while an array uses it
        # re-entrant: a block's finaliser (_release) may run inside empty() on the same thread, when
        # an allocation there triggers the cyclic collector and it frees an array of this pool
        self._lock = threading.RLock()

    def empty(self, shape, dtype=np.float64) -> np.ndarray:
        dt = np.dtype(dtype)
        count = int(np.prod(shape))
        n = max(count * dt.itemsize, 1)
        block = None
        with self._lock:
            fits = [i for i, b in enumerate(self._free) if n <= b.nbytes <= 2 * n]
            if fits:
                block = self._free.pop(min(fits, key=lambda i: self._free[i].nbytes))
        if block is None:
            block = np.empty(n, np.uint8)
        proxy = (ctypes.c_char * block.nbytes).from_address(block.ctypes.data)
        key = id(proxy)
        with self._lock:
            self._busy[key] = block
        weakref.finalize(proxy, self._release, key)
        return np.frombuffer(proxy, dt, count).reshape(shape)

    def _release(self, key):
        with self._lock:
            block = self._busy.pop(key, None)
            if block is not None and sum(b.nbytes for b in self._free) + block.nbytes <= self.cap:
                self._free.append(block)

    def idle_bytes(self) -> int:
        with self._lock:
            return sum(b.nbytes for b in self._free)

    def clear(self):
        """Release every idle block (blocks still behind live arrays return to the pool later)."""
        with self._lock:
            self._free = []


_host_pool: "HostPool | None" = None


def host_pool() -> HostPool:
    global _host_pool
    if _host_pool is None:
        _host_pool = HostPool()
    return _host_pool


class DeviceBuffer:
    """Raw HBM allocation owned by a context (e.g. a device-resident (N,4) float64 AoS cloud)."""

    def __init__(self, ctx: Context, nbytes: int):
        self.ctx, self.lib, self.nbytes = ctx, ctx.lib, int(nbytes)
        p = c_void_p()
        check(self.lib.mc_device_alloc(ctx.handle, self.nbytes, ctypes.byref(p)), "device_alloc")
        self.ptr = p
        self._fin = weakref.finalize(self, self.lib.mc_device_free, ctx.handle, p)

    def close(self):
        self._fin()

    def to_host(self, dtype=np.float64, shape=None, count=None) -> np.ndarray:
        n = self.nbytes // np.dtype(dtype).itemsize
        out = np.empty(n if count is None else min(int(count), n), dtype)
        check(self.lib.mc_memcpy_d2h(self.ctx.handle, out.ctypes.data_as(c_void_p), self.ptr, out.nbytes), "d2h")
        return out.reshape(shape) if shape is not None else out

    def from_host(self, a: np.ndarray):
        a = np.ascontiguousarray(a)
        if a.nbytes > self.nbytes:
            raise ValueError("array larger than the device buffer")
        check(self.lib.mc_memcpy_h2d(self.ctx.handle, self.ptr, a.ctypes.data_as(c_void_p), a.nbytes), "h2d")


class Batch:
    """Device-resident ragged frame batch (blocked CSR: 256-point blocks of float32 columns in HBM)."""

    def __init__(self, ctx: Context, counts, with_time: bool = False, with_pcd_len: bool = False):
        self.ctx = ctx
        self.lib = ctx.lib
        self.counts = np.ascontiguousarray(np.atleast_1d(counts), dtype=np.int64)
        if self.counts.ndim != 1 or (self.counts < 0).any():
            raise ValueError("counts must be a 1-D array of non-negative frame sizes")
        self.with_time = bool(with_time)
        self.with_pcd_len = bool(with_pcd_len)
        h = c_void_p()
        # with_pcd_len: the kernels that write the columns also keep each block's ASCII PCD text
        # length, so encode_pcd_batch needs no measure pass (include/mcdeskew.h MC_BATCH_WITH_PCD_LEN)
        flags = (_lib.MC_BATCH_WITH_TIME if with_time else 0) | (_lib.MC_BATCH_WITH_PCD_LEN if with_pcd_len else 0)
        check(self.lib.mc_batch_create(ctx.handle, len(self.counts), ptr(self.counts, c_int64), flags,
                                       ctypes.byref(h)), "batch_create")
        self.handle = h
        self._fin = weakref.finalize(self, self.lib.mc_batch_destroy, h)
        n, p = c_int64(), c_int64()
        f, t = c_int32(), c_int32()
        check(self.lib.mc_batch_info(h, ctypes.byref(n), ctypes.byref(p), ctypes.byref(f), ctypes.byref(t)))
        self.n_points, self.padded_points, self.n_frames, self.n_tiles = n.value, p.value, f.value, t.value
        self.offsets = np.concatenate([[0], np.cumsum(self.counts)]).astype(np.int64)

    def close(self):
        self._fin()

    def pcd_len_current(self) -> bool:
        """True when the per-block PCD text sums describe the current columns."""
        v = c_int32()
        check(self.lib.mc_batch_pcd_len_current(self.handle, ctypes.byref(v)), "pcd_len_current")
        return bool(v.value)

    def padded_offsets(self) -> np.ndarray:
        o = np.zeros(self.n_frames + 1, np.int64)
        check(self.lib.mc_batch_padded_offsets(self.handle, ptr(o, c_int64)))
        return o

    def set_frame_times(self, t_frame):
        t = _f64(np.atleast_1d(t_frame))
        if len(t) != self.n_frames:
            raise ValueError("one frame time per frame expected")
        check(self.lib.mc_batch_set_frame_times(self.handle, ptr(t, c_double)), "set_frame_times")

    def set_frame_starts(self, start_ns):
        s = np.ascontiguousarray(np.atleast_1d(start_ns), dtype=np.int64)
        if len(s) != self.n_frames:
            raise ValueError("one frame start per frame expected")
        check(self.lib.mc_batch_set_frame_start_ns(self.handle, ptr(s, c_int64)), "set_frame_starts")

    # ---- host <-> device ----------------------------------------------------------------
    def upload_aos(self, points):
        """Dense (N, ld>=4) float64 AoS — the reference's (N,4) [x,y,z,intensity] layout (LMC:770)."""
        a = np.ascontiguousarray(points, dtype=np.float64)
        if a.ndim != 2:
            raise IndexError("too many indices for array: points must be 2-D (N, 4)")
        if a.shape[0] != self.n_points:
            raise ValueError(f"batch holds {self.n_points} points, got {a.shape[0]}")
        check(self.lib.mc_batch_upload_aos_f64(self.handle, ptr(a, c_double), a.shape[1]), "upload_aos")

    def upload_columns(self, x=None, y=None, z=None, intensity=None):
        cols = []
        for c in (x, y, z, intensity):
            if c is None:
                cols.append(None)
                continue
            c = np.ascontiguousarray(c, dtype=np.float32)
            if c.shape != (self.n_points,):
                raise ValueError(f"column of {self.n_points} points expected, got {c.shape}")
            cols.append(c)
        check(self.lib.mc_batch_upload_columns_f32(self.handle, *[ptr(c, c_float) for c in cols]), "upload_columns")

    def upload_time(self, t_ns):
        t = np.asarray(t_ns)
        if t.shape != (self.n_points,):
            raise ValueError(f"t_ns of {self.n_points} points expected, got {t.shape}")
        if t.size and (t.min() < -2**31 or t.max() > 2**31 - 1):
            raise ValueError("t_ns (time since frame start) must fit in int32 nanoseconds (+-2.147 s)")
        t = np.ascontiguousarray(t, dtype=np.int32)
        check(self.lib.mc_batch_upload_time_ns(self.handle, ptr(t, c_int32)), "upload_time")

    def stage_aos_device(self, buf: "DeviceBuffer", ld: int = 4):
        """Device-resident dense (N, ld) float64 AoS -> this batch's columns (async, in HBM)."""
        if buf.nbytes < self.n_points * ld * 8:
            raise ValueError("device buffer smaller than the batch's AoS")
        check(self.lib.mc_batch_stage_aos_f64_device(self.handle, buf.ptr, int(ld)), "stage_aos_device")

    def fetch_aos_device(self, buf: "DeviceBuffer"):
        """This batch's columns -> device-resident dense (N,4) float64 AoS (async, in HBM)."""
        if buf.nbytes < self.n_points * 32:
            raise ValueError("device buffer smaller than the batch's (N,4) float64 AoS")
        check(self.lib.mc_batch_fetch_aos_f64_device(self.handle, buf.ptr), "fetch_aos_device")

    def download_aos(self) -> np.ndarray:
        out = np.empty((self.n_points, 4), np.float64)
        check(self.lib.mc_batch_download_aos_f64(self.handle, ptr(out, c_double)), "download_aos")
        return out

    def download_frames(self, f0: int, f1: int) -> np.ndarray:
        """Frames [f0, f1) as dense (n, 4) float64 rows (a spot check of a batch too large to
        bring back whole)."""
        f0, f1 = int(f0), int(f1)
        if not 0 <= f0 <= f1 <= self.n_frames:
            raise ValueError(f"frame range [{f0}, {f1}) outside [0, {self.n_frames})")
        out = np.empty((int(self.offsets[f1] - self.offsets[f0]), 4), np.float64)
        check(self.lib.mc_batch_download_frames_aos_f64(self.handle, f0, f1, ptr(out, c_double)), "download_frames")
        return out

    def download_columns(self):
        cols = [np.empty(self.n_points, np.float32) for _ in range(4)]
        check(self.lib.mc_batch_download_columns_f32(self.handle, *[ptr(c, c_float) for c in cols]),
              "download_columns")
        return tuple(cols)

    def download_time(self) -> np.ndarray:
        t = np.empty(self.n_points, np.int32)
        check(self.lib.mc_batch_download_time_ns(self.handle, ptr(t, c_int32)), "download_time")
        return t

    def synth(self, seed: int = 0, frame_id_base: int = 1000):
        """Fill with synthetic Mid-70 frames on the device (bit-identical to oracle/synth.py)."""
        check(self.lib.mc_batch_synth(self.handle, int(seed) % 2**64, int(frame_id_base)), "synth")

    def checksum(self) -> np.ndarray:
        s = np.zeros(5, np.float64)
        check(self.lib.mc_batch_checksum(self.handle, ptr(s, c_double)), "checksum")
        return s

    def split(self, aos: np.ndarray) -> list:
        """Split a dense (N,4) array into per-frame arrays (frame order)."""
        return [aos[self.offsets[f]:self.offsets[f + 1]] for f in range(self.n_frames)]


def deskew_points_f64(ctx: Context, mode: str, counts, points, t_ns, frame_times=None, frame_start_ns=None) -> np.ndarray:
    """The per-point modes on host float64 rows (mc_deskew_points_f64): frames back to back
    (``counts``), ``points`` (N, >=3) float64, ``t_ns`` (N,) int64 ns since each point's frame start,
    ``frame_times`` (SLERP, s) or ``frame_start_ns`` (IMU) per frame.  Returns (N, 4) float64:
    x', y', z' in float64, column 3 = points[:, 3] (0 for 3-column input).  The pose / IMU table is
    the one uploaded to ``ctx``."""
    c = np.ascontiguousarray(np.atleast_1d(counts), dtype=np.int64)
    p = np.asarray(points)
    if p.ndim != 2:
        raise IndexError(f"too many indices for array: array is {p.ndim}-dimensional, but 2 were indexed")
    p = np.ascontiguousarray(p, dtype=np.float64)
    t = np.ascontiguousarray(t_ns, dtype=np.int64).reshape(-1)
    n = int(c.sum())
    if p.shape[0] != n or t.shape[0] != n:
        raise ValueError(f"counts add up to {n} points; got {p.shape[0]} rows and {t.shape[0]} timestamps")
    ft = None if frame_times is None else np.ascontiguousarray(frame_times, dtype=np.float64)
    fs = None if frame_start_ns is None else np.ascontiguousarray(frame_start_ns, dtype=np.int64)
    for v, what in ((ft, "frame_times"), (fs, "frame_start_ns")):
        if v is not None and v.shape != (len(c),):
            raise ValueError(f"{what}: one value per frame expected ({len(c)}), got {v.shape}")
    out = np.empty((n, 4), np.float64)
    check(ctx.lib.mc_deskew_points_f64(ctx.handle, _lib.MODES[mode], len(c), ptr(c, c_int64), ptr(p, c_double),
                                       p.shape[1], ptr(t, c_int64), ptr(ft, c_double),
                                       ptr(fs, c_int64), ptr(out, c_double)), f"deskew_points_f64[{mode}]")
    return out


_default_ctx: Context | None = None


def default_context() -> Context:
    """Process-wide context used by the drop-in reference-compatible functions."""
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context()
    return _default_ctx
