"""CPU restatement of the reference's output codecs (numpy, vectorised) — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may import this
module, as the checker / timed CPU baseline.  Parity: PINNED byte for byte against files written by
the reference itself (tests/golden/codecs.npz, made by tests/golden/make_golden.py::make_codecs).

LVX v1.1 (LMC:24-272, LivoxLVXWriter.write_compatible_lvx):
  file   = public header 24 B (16 B signature "livox_tech", version 1.1.0.0, magic 0xAC0EA767)
           + private header 5 B (frame duration 50 ms u32, device count 1)      LMC:86-110
           + device info 59 B (LiDAR SN, hub SN, index, type 1, extrinsics off)  LMC:146-172
  frame  = 24 B header (own offset, next offset or 0 for the last, frame_id)     LMC:174-193
           + ceil(n/96) packages                                                 LMC:196-199
  package= 22 B header (ver 5, slot 0, lidar 1, ts type 1, data type 2, timestamp ns u64)
           + 96 records of 14 B, zero-padded                                     LMC:201-250
  record = int32 trunc(clip(x*1000)) x,y,z (mm), u8 trunc(clip(i*255, 0, 255)) (128 without an
           intensity column), tag 0                                              LMC:252-272
ASCII PCD v0.7 (LMC:932-948): 11 header lines, then "%.6f %.6f %.6f %.6f\\n" per point with
Python's correctly rounded float formatting.
"""
from __future__ import annotations

import struct

import numpy as np

LVX_PKG_POINTS = 96
LVX_REC = 14
LVX_PKG_HDR = 22
LVX_PKG = LVX_PKG_HDR + LVX_PKG_POINTS * LVX_REC
LVX_FRAME_HDR = 24


def lvx_file_header() -> bytes:
    """The 88 constant bytes ahead of the first frame (LMC:86-110, 146-172)."""
    pub = b"livox_tech" + bytes(6) + bytes([1, 1, 0, 0]) + struct.pack("<I", 0xAC0EA767)
    priv = struct.pack("<IB", 50, 1)
    dev = b"3GGDJ6K00200101\x00" + bytes(16) + bytes([0, 1, 0]) + bytes(24)
    return pub + priv + dev


def lvx_frame_positions(counts) -> np.ndarray:
    """Byte offset of every frame (LMC:115-132) plus the file size as the last entry."""
    counts = np.asarray(counts, np.int64)
    sizes = LVX_FRAME_HDR + (counts + LVX_PKG_POINTS - 1) // LVX_PKG_POINTS * LVX_PKG
    return len(lvx_file_header()) + np.concatenate([[0], np.cumsum(sizes)])


def _records(points: np.ndarray) -> np.ndarray:
    n = len(points)
    rec = np.zeros((n, LVX_REC), np.uint8)
    if n == 0:
        return rec
    xyz = np.clip(points[:, :3] * 1000, -2147483648, 2147483647)
    if np.isnan(xyz).any():
        raise ValueError("cannot convert float NaN to integer")
    rec[:, :12] = np.trunc(xyz).astype("<i4").view(np.uint8).reshape(n, 12)
    if points.shape[1] > 3:
        refl = np.clip(points[:, 3] * 255, 0, 255)
        if np.isnan(refl).any():
            raise ValueError("cannot convert float NaN to integer")
        rec[:, 12] = np.trunc(refl).astype(np.uint8)
    else:
        rec[:, 12] = 128
    return rec


def lvx_bytes(frames) -> bytes:
    """frames: sequence of dicts with frame_id, timestamp (s), points (n, >=3)."""
    pos = lvx_frame_positions([len(f["points"]) for f in frames])
    parts = [lvx_file_header()]
    for i, fr in enumerate(frames):
        nxt = int(pos[i + 1]) if i + 1 < len(frames) else 0
        parts.append(struct.pack("<QQQ", int(pos[i]), nxt, int(fr["frame_id"])))
        pts = np.asarray(fr["points"], np.float64)
        rec = _records(pts)
        npkg = (len(pts) + LVX_PKG_POINTS - 1) // LVX_PKG_POINTS
        body = np.zeros((npkg, LVX_PKG), np.uint8)
        hdr = bytes([0, 5, 0, 1, 0, 0, 0, 0, 0, 1, 2, 0, 0, 0]) + struct.pack("<Q", int(fr["timestamp"] * 1e9))
        body[:, :LVX_PKG_HDR] = np.frombuffer(hdr, np.uint8)
        padded = np.zeros((npkg * LVX_PKG_POINTS, LVX_REC), np.uint8)
        padded[:len(pts)] = rec
        body[:, LVX_PKG_HDR:] = padded.reshape(npkg, LVX_PKG_POINTS * LVX_REC)
        parts.append(body.tobytes())
    return b"".join(parts)


def pcd_header(n: int) -> str:
    return ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z intensity\n"
            "SIZE 4 4 4 4\nTYPE F F F F\nCOUNT 1 1 1 1\n"
            f"WIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\nDATA ascii\n")


def pcd_ascii_bytes(points) -> bytes:
    pts = np.asarray(points, np.float64).reshape(-1, np.shape(points)[-1] if np.ndim(points) == 2 else 4)
    body = "".join("%s %s %s %s\n" % tuple(format(float(v), ".6f") for v in row[:4]) for row in pts)
    return (pcd_header(len(pts)) + body).encode("ascii")
