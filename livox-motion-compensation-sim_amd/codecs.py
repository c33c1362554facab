"""Output codecs on the device: LVX v1.1 (LMC:24-272) and ASCII PCD (LMC:932-948), byte-exact.

The reference's writers loop over points in Python (``struct.pack`` per 14-byte record, an
f-string per PCD line).  Here the point records / text lines are produced by gfx950 kernels from a
device-resident (N, ld) float64 cloud (include/mcdeskew.h ``mc_lvx_encode`` / ``mc_pcd_encode``);
the host only adds the constant headers and writes the bytes.

  LivoxLVXWriter.write_compatible_lvx(filename, frames_data)   LMC:57-143 (same validation,
                                                                True / False result)
  save_pcd(points, filename)                                   LMC:932-948
  encode_lvx / encode_pcd / encode_pcd_frames                  the bytes, without a file
  encode_lvx_batch / encode_pcd_batch                          straight from a device Batch
  deskew_pcd_batch / deskew_pcd_frames                         deskew -> PCD lines, the deskew
                                                                kernel measuring the text (no
                                                                separate measure pass)
"""
from __future__ import annotations

import ctypes
from ctypes import c_double, c_int64, c_uint8, c_uint64, c_void_p
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check, ptr
from .runtime import Batch, Context, DeviceBuffer, default_context

PCD_HEADER = ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z intensity\n"
              "SIZE 4 4 4 4\nTYPE F F F F\nCOUNT 1 1 1 1\nWIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\n"
              "POINTS {n}\nDATA ascii\n")   # LMC:935-945


def pcd_header(n: int) -> bytes:
    return PCD_HEADER.format(n=int(n)).encode("ascii")


def lvx_layout(counts) -> np.ndarray:
    """Byte offset of every frame in the LVX file (LMC:113-132); the last entry is the file size."""
    counts = np.ascontiguousarray(counts, dtype=np.int64)
    pos = np.zeros(len(counts) + 1, np.int64)
    lib = _lib.load()
    check(lib.mc_lvx_layout(len(counts), ptr(counts, c_int64), ptr(pos, c_int64)), "lvx_layout")
    return pos


def _device_cloud(ctx: Context, frames: Sequence[np.ndarray], min_cols: int):
    """Frames stacked back to back into one device (N, 4) float64 buffer (columns beyond the 4th
    are dropped, a 3-column frame gets a zero 4th column) + counts + per-frame 'has intensity'."""
    counts = np.array([len(f) for f in frames], np.int64)
    n = int(counts.sum())
    aos = np.zeros((n, 4), np.float64)
    has = np.ones(len(frames), np.uint8)
    o = 0
    for i, f in enumerate(frames):
        f = np.asarray(f)
        if f.ndim != 2 or f.shape[1] < min_cols:
            raise IndexError(f"frame {i}: points need at least {min_cols} columns, got shape {f.shape}")
        k = min(f.shape[1], 4)
        aos[o:o + len(f), :k] = f[:, :k]
        has[i] = f.shape[1] > 3
        o += len(f)
    buf = ctx.device_buffer(max(aos.nbytes, 8))
    if n:
        buf.from_host(aos)
    return buf, counts, has


# ---- LVX v1.1 --------------------------------------------------------------------------------
def _lvx_encode_device(ctx: Context, d_aos, ld, counts, frame_ids, ts_ns, has) -> np.ndarray:
    counts = np.ascontiguousarray(counts, np.int64)
    pos = lvx_layout(counts)
    size = int(pos[-1])
    ids = np.ascontiguousarray(frame_ids, np.uint64)
    ts = np.ascontiguousarray(ts_ns, np.uint64)
    hasp = None if has is None else ptr(np.ascontiguousarray(has, np.uint8), c_uint8)
    out = ctx.device_buffer(size)
    try:
        check(ctx.lib.mc_lvx_encode(ctx.handle, d_aos, int(ld), len(counts), ptr(counts, c_int64),
                                    ptr(ids, c_uint64), ptr(ts, c_uint64), hasp, out.ptr, size), "lvx_encode")
        return out.to_host(np.uint8)
    finally:
        out.close()


def _u64(v, what):
    v = int(v)
    if not 0 <= v < 2 ** 64:
        raise ValueError(f"{what} {v} does not fit the LVX u64 field")   # struct.error in LMC:183-191
    return v


def encode_lvx(frames_data: List[dict], context: Context | None = None) -> bytes:
    """The bytes write_compatible_lvx (LMC:57-143) writes for ``frames_data`` (dicts with
    frame_id, timestamp (s), points (n, >=3)).  NaN coordinates raise ValueError."""
    ctx = context or default_context()
    frames = [np.asarray(fd["points"], np.float64) for fd in frames_data]
    ids = [_u64(fd["frame_id"], "frame_id") for fd in frames_data]
    ts = [_u64(int(fd["timestamp"] * 1e9), "timestamp_ns") for fd in frames_data]   # LMC:176
    buf, counts, has = _device_cloud(ctx, frames, 3)
    try:
        return _lvx_encode_device(ctx, buf.ptr, 4, counts, ids, ts, has).tobytes()
    finally:
        buf.close()


def encode_lvx_device_rows(rows: DeviceBuffer, counts, frames_data: List[dict]) -> bytes:
    """encode_lvx of ``frames_data`` whose points are already on the device as (N, 4) float64 rows,
    frames back to back (``counts``): no host staging or upload (save_lvx after simulate_frames)."""
    ids = [_u64(fd["frame_id"], "frame_id") for fd in frames_data]
    ts = [_u64(int(fd["timestamp"] * 1e9), "timestamp_ns") for fd in frames_data]   # LMC:176
    return _lvx_encode_device(rows.ctx, rows.ptr, 4, counts, ids, ts, None).tobytes()


def encode_lvx_batch(batch: Batch, frame_ids, timestamps) -> bytes:
    """LVX file of a device batch's frames, encoded from the batch's float32 columns in HBM
    (mc_lvx_encode_batch): the records of the reference writer applied to ``batch.download_aos()``."""
    ctx = batch.ctx
    if len(frame_ids) != batch.n_frames or len(timestamps) != batch.n_frames:
        raise ValueError("one frame id and one timestamp per frame expected")
    ids = np.array([_u64(i, "frame_id") for i in frame_ids], np.uint64)
    ts = np.array([_u64(int(t * 1e9), "timestamp_ns") for t in timestamps], np.uint64)
    size = int(lvx_layout(batch.counts)[-1])
    out = ctx.device_buffer(size)
    try:
        check(ctx.lib.mc_lvx_encode_batch(ctx.handle, batch.handle, ptr(ids, c_uint64), ptr(ts, c_uint64), out.ptr,
                                          size), "lvx_encode_batch")
        return out.to_host(np.uint8).tobytes()
    finally:
        out.close()


class LivoxLVXWriter:
    """Drop-in for lidar_motion_compensation.LivoxLVXWriter (LMC:24-272); the constants are the
    reference's (LMC:38-55), the packing runs on the GPU."""

    def __init__(self, context: Context | None = None):
        self.LVX_FILE_SIGNATURE = b"livox_tech" + bytes(6)
        self.MAGIC_CODE = 0xAC0EA767
        self.DEVICE_TYPE_MID70 = 1
        self.FRAME_DURATION_MS = 50
        self.DATA_TYPE_CARTESIAN = 2
        self.POINTS_PER_PACKAGE = 96
        self.PACKAGE_VERSION = 5
        self.SLOT_ID = 0
        self.LIDAR_ID = 1
        self.TIMESTAMP_TYPE = 1
        self._context = context

    def write_compatible_lvx(self, filename: str, frames_data: List[dict]) -> bool:
        return self._write(filename, frames_data, lambda: encode_lvx(frames_data, self._context))

    def _write(self, filename: str, frames_data: List[dict], encode) -> bool:
        # LMC:70-77: argument validation raises; any failure after it returns False
        if not filename or not isinstance(filename, str):
            raise ValueError("Invalid filename provided")
        if not frames_data or not isinstance(frames_data, list):
            raise ValueError("Invalid frames_data provided")
        try:
            print(f"Writing LVX file: {filename}")
            with open(filename, "wb") as f:
                data = encode()
                f.write(data)
            print(f"✅ LVX file created successfully: {len(data):,} bytes")
            return True
        except Exception as e:   # LMC:141-143
            print(f"❌ Error writing LVX file: {e}")
            return False


# ---- ASCII PCD -------------------------------------------------------------------------------
def _pcd_encode_device(ctx: Context, d_aos, ld, counts) -> List[bytes]:
    """Per cloud the PCD header + point lines."""
    counts = np.ascontiguousarray(counts, np.int64)
    return [pcd_header(c) + body for c, body in zip(counts, _pcd_bodies_device(ctx, d_aos, ld, counts))]


def _pcd_bodies_device(ctx: Context, d_aos, ld, counts) -> List[bytes]:
    """Per cloud its point lines only (LMC:946-948)."""
    counts = np.ascontiguousarray(counts, np.int64)
    F = len(counts)
    pos = np.zeros(F + 1, np.int64)
    cap = max(int(counts.sum()) * 48, 64)
    for _ in range(2):
        out = ctx.device_buffer(cap)
        try:
            rc = ctx.lib.mc_pcd_encode(ctx.handle, d_aos, int(ld), F, ptr(counts, c_int64), out.ptr, cap,
                                       ptr(pos, c_int64))
            if rc == _lib.MC_ERR_SPACE:
                cap = int(pos[-1])        # exact size now known: one more pass
                continue
            check(rc, "pcd_encode")
            text = out.to_host(np.uint8, count=int(pos[-1])).tobytes() if pos[-1] else b""
        finally:
            out.close()
        return [text[pos[f]:pos[f + 1]] for f in range(F)]
    raise _lib.McError("pcd_encode: output size changed between passes")


def encode_pcd_frames(clouds: Sequence[np.ndarray], context: Context | None = None) -> List[bytes]:
    """Per cloud, the bytes save_pcd (LMC:932-948) writes; all clouds in one launch pair."""
    ctx = context or default_context()
    buf, counts, _ = _device_cloud(ctx, [np.asarray(c, np.float64) for c in clouds], 4)
    try:
        return _pcd_encode_device(ctx, buf.ptr, 4, counts)
    finally:
        buf.close()


def encode_pcd_bodies(clouds: Sequence[np.ndarray], context: Context | None = None) -> List[bytes]:
    """Per cloud its point lines without the header (merged files reuse the frames' lines)."""
    ctx = context or default_context()
    buf, counts, _ = _device_cloud(ctx, [np.asarray(c, np.float64) for c in clouds], 4)
    try:
        return _pcd_bodies_device(ctx, buf.ptr, 4, counts)
    finally:
        buf.close()


def encode_pcd_bodies_device_rows(rows: DeviceBuffer, counts) -> List[bytes]:
    """encode_pcd_bodies of clouds already on the device as (N, 4) float64 rows, back to back."""
    return _pcd_bodies_device(rows.ctx, rows.ptr, 4, counts)


def encode_pcd(points, context: Context | None = None) -> bytes:
    return encode_pcd_frames([points], context)[0]


def encode_pcd_batch(batch: Batch) -> List[bytes]:
    """PCD bytes of every frame of a device batch, formatted from the batch's float32 columns in HBM
    (mc_pcd_encode_batch): the reference writer applied to the values widened to float64."""
    ctx = batch.ctx
    counts = np.ascontiguousarray(batch.counts, np.int64)
    F = len(counts)
    pos = np.zeros(F + 1, np.int64)
    cap = max(int(counts.sum()) * 48, 64)
    for _ in range(2):
        out = ctx.device_buffer(cap)
        try:
            rc = ctx.lib.mc_pcd_encode_batch(ctx.handle, batch.handle, out.ptr, cap, ptr(pos, c_int64))
            if rc == _lib.MC_ERR_SPACE:
                cap = int(pos[-1])
                continue
            check(rc, "pcd_encode_batch")
            text = out.to_host(np.uint8, count=int(pos[-1])).tobytes() if pos[-1] else b""
        finally:
            out.close()
        return [pcd_header(c) + text[pos[f]:pos[f + 1]] for f, c in enumerate(counts)]
    raise _lib.McError("pcd_encode_batch: output size changed between passes")


def deskew_pcd_batch(inp: Batch, out: Batch, mode: str = "frame", pose_select: str = "searchsorted",
                     text=None):
    """Deskew ``inp`` into ``out`` and write out's ASCII PCD point lines, both on the device
    (mc_deskew_pcd: the deskew kernel sums each block's text bytes, so the writer needs no measure
    pass over ``out``) — LMC:831 -> 887-889 -> 932-948 on device-resident frames.  Returns
    (device text buffer, body_pos) with frame f's lines at [body_pos[f], body_pos[f+1]); ``text``: a
    DeviceBuffer to reuse.  The buffer is sized for the longest packed line (52 bytes: four values of
    "-dddd.dddddd" and their separators), so the packed path never needs a second pass; a ``text``
    smaller than that, or text of lines beyond the packed path that still does not fit, is closed
    and replaced by a new buffer (the returned one) of exactly the size the first pass reported."""
    ctx = inp.ctx
    if out is inp:
        raise ValueError("deskew_pcd needs an output batch other than the input")
    counts = np.ascontiguousarray(out.counts, np.int64)
    pos = np.zeros(len(counts) + 1, np.int64)
    cap = max(int(counts.sum()) * 52, 64)     # the packed maximum: 4 x (1 + 4 + 7) + 4
    if text is None or text.nbytes < cap:
        if text is not None:
            text.close()
        text = ctx.device_buffer(cap)
    rc = ctx.lib.mc_deskew_pcd(ctx.handle, inp.handle, out.handle, _lib.MODES[mode], _lib.POSE_SELECT[pose_select],
                               text.ptr, text.nbytes, ptr(pos, c_int64))
    if rc == _lib.MC_ERR_SPACE:   # out is deskewed: the plain writer with the size it reported
        text.close()
        text = ctx.device_buffer(int(pos[-1]))
        rc = ctx.lib.mc_pcd_encode_batch(ctx.handle, out.handle, text.ptr, text.nbytes, ptr(pos, c_int64))
    check(rc, f"deskew_pcd[{mode}]")
    return text, pos


def deskew_pcd_frames(inp: Batch, out: Batch, mode: str = "frame", pose_select: str = "searchsorted") -> List[bytes]:
    """:func:`deskew_pcd_batch` with each frame's whole PCD file (header + lines) on the host."""
    text, pos = deskew_pcd_batch(inp, out, mode, pose_select)
    try:
        body = text.to_host(np.uint8, count=int(pos[-1])).tobytes() if pos[-1] else b""
    finally:
        text.close()
    return [pcd_header(int(c)) + body[pos[f]:pos[f + 1]] for f, c in enumerate(out.counts)]


def save_pcd(points, filename: str, context: Context | None = None) -> None:
    """LMC:932-948: ASCII PCD v0.7 with x y z intensity; fewer than 4 columns -> IndexError."""
    pts = np.asarray(points)
    if pts.ndim != 2:
        raise IndexError(f"points must be 2-dimensional, got shape {pts.shape}")
    data = encode_pcd(pts, context) if len(pts) else pcd_header(0)
    with open(filename, "wb") as f:
        f.write(data)
