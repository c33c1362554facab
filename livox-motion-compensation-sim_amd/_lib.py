"""ctypes binding of libmcdeskew.so (the C-ABI in include/mcdeskew.h).

The library is the product: there is no CPU fallback.  If it is missing, or no gfx950 GPU is
visible, every entry point raises ``McLibraryError`` — it never degrades silently.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char, c_char_p, c_double, c_int, c_int32, c_int64, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MCDESKEW_LIB", os.path.join(_HERE, "libmcdeskew.so"))

MC_OK = 0
MC_ERR_INVALID = -1
MC_ERR_HIP = -2
MC_ERR_NOMEM = -3
MC_ERR_STATE = -4
MC_ERR_INDEX = -5
MC_ERR_COMM = -6
MC_ERR_SPACE = -7

MC_MODE_FRAME = 0
MC_MODE_POSE_SLERP = 1
MC_MODE_IMU = 2
MC_POSE_SEARCHSORTED = 0
MC_POSE_DIRECT = 1
MC_BATCH_WITH_TIME = 1
MC_BATCH_WITH_PCD_LEN = 2

MODES = {"frame": MC_MODE_FRAME, "pose_slerp": MC_MODE_POSE_SLERP, "imu": MC_MODE_IMU}
POSE_SELECT = {"searchsorted": MC_POSE_SEARCHSORTED, "direct": MC_POSE_DIRECT}


class McError(RuntimeError):
    """A HIP / RCCL / state failure inside libmcdeskew."""


class McLibraryError(ImportError):
    """libmcdeskew.so is missing or unusable: the HIP path cannot run (no silent fallback)."""


_pd = POINTER(c_double)
_pi64 = POINTER(c_int64)
_pi32 = POINTER(c_int32)
_pf = POINTER(ctypes.c_float)

# name -> (restype, argtypes)
_SIGS = {
    "mc_abi_version": (c_int, []),
    "mc_last_error": (c_char_p, []),
    "mc_device_count": (c_int, [POINTER(c_int)]),
    "mc_device_pci_bus_id": (c_int, [c_int, POINTER(c_char), c_int]),
    "mc_create": (c_int, [c_int, POINTER(c_void_p)]),
    "mc_destroy": (c_int, [c_void_p]),
    "mc_sync": (c_int, [c_void_p]),
    "mc_set_trajectory": (c_int, [c_void_p, c_int64, _pd, _pd, _pd]),
    "mc_set_imu": (c_int, [c_void_p, c_int64, _pi64, _pd]),
    "mc_batch_create": (c_int, [c_void_p, c_int32, _pi64, c_uint32, POINTER(c_void_p)]),
    "mc_batch_destroy": (c_int, [c_void_p]),
    "mc_batch_info": (c_int, [c_void_p, _pi64, _pi64, _pi32, _pi32]),
    "mc_batch_padded_offsets": (c_int, [c_void_p, _pi64]),
    "mc_batch_pcd_len_current": (c_int, [c_void_p, _pi32]),
    "mc_batch_set_frame_times": (c_int, [c_void_p, _pd]),
    "mc_batch_set_frame_start_ns": (c_int, [c_void_p, _pi64]),
    "mc_batch_upload_aos_f64": (c_int, [c_void_p, _pd, c_int64]),
    "mc_batch_upload_columns_f32": (c_int, [c_void_p, _pf, _pf, _pf, _pf]),
    "mc_batch_upload_time_ns": (c_int, [c_void_p, _pi32]),
    "mc_batch_download_aos_f64": (c_int, [c_void_p, _pd]),
    "mc_batch_download_frames_aos_f64": (c_int, [c_void_p, c_int32, c_int32, _pd]),
    "mc_batch_download_columns_f32": (c_int, [c_void_p, _pf, _pf, _pf, _pf]),
    "mc_batch_download_time_ns": (c_int, [c_void_p, _pi32]),
    "mc_device_alloc": (c_int, [c_void_p, c_int64, POINTER(c_void_p)]),
    "mc_device_free": (c_int, [c_void_p, c_void_p]),
    "mc_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_void_p, c_int64]),
    "mc_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_void_p, c_int64]),
    "mc_memcpy_d2d": (c_int, [c_void_p, c_void_p, c_void_p, c_int64]),
    "mc_batch_stage_aos_f64_device": (c_int, [c_void_p, c_void_p, c_int64]),
    "mc_batch_fetch_aos_f64_device": (c_int, [c_void_p, c_void_p]),
    "mc_timing_read_layout": (c_int, [c_void_p, _pd, _pi64]),
    "mc_set_environment": (c_int, [c_void_p, c_int64, _pd, c_int64]),
    "mc_scan_count": (c_int, [c_void_p, c_int32, _pd, c_int, _pd, c_int64, _pi64]),
    "mc_scan_emit": (c_int, [c_void_p, c_void_p, _pd]),
    "mc_scan_emit_f64": (c_int, [c_void_p, _pd, c_void_p, c_void_p]),
    "mc_timing_read_scan": (c_int, [c_void_p, _pd, _pi64]),
    "mc_lvx_layout": (c_int, [c_int32, _pi64, _pi64]),
    "mc_lvx_encode": (c_int, [c_void_p, c_void_p, c_int64, c_int32, _pi64, POINTER(c_uint64), POINTER(c_uint64),
                              POINTER(ctypes.c_uint8), c_void_p, c_int64]),
    "mc_pcd_encode": (c_int, [c_void_p, c_void_p, c_int64, c_int32, _pi64, c_void_p, c_int64, _pi64]),
    "mc_lvx_encode_batch": (c_int, [c_void_p, c_void_p, POINTER(c_uint64), POINTER(c_uint64), c_void_p, c_int64]),
    "mc_pcd_encode_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, _pi64]),
    "mc_deskew_pcd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int64, _pi64]),
    "mc_timing_read_codec": (c_int, [c_void_p, _pd, _pi64]),
    "mc_batch_synth": (c_int, [c_void_p, c_uint64, c_int64]),
    "mc_batch_checksum": (c_int, [c_void_p, _pd]),
    "mc_deskew": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int]),
    "mc_deskew_steps": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int32, c_int32]),
    "mc_tune_order": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int32, c_int32, _pd, _pi32]),
    "mc_transform_affine": (c_int, [c_void_p, c_void_p, c_void_p, c_int32, _pd, c_int]),
    "mc_transform_pointcloud_f64": (c_int, [c_void_p, _pd, c_int64, c_int64, _pd, _pd, _pd]),
    "mc_rotation_from_euler_xyz": (c_int, [c_int64, _pd, _pd]),
    "mc_affine_rows_f64": (c_int, [c_void_p, c_int32, _pi64, _pd, c_int64, c_int32, _pd, c_int, _pd]),
    "mc_deskew_points_f64": (c_int, [c_void_p, c_int, c_int32, _pi64, _pd, c_int64, _pi64, _pd, _pi64, _pd]),
    # frames / outs: arrays of row pointers (passed as the address of a uintp array)
    "mc_align_frames_host_f64": (c_int, [c_void_p, c_int32, c_void_p, _pi64, _pi64, _pd, c_int, c_void_p]),
    "mc_timing_enable": (c_int, [c_void_p, c_int]),
    "mc_timing_read": (c_int, [c_void_p, _pd, _pi64, _pd, _pi64]),
    "mc_timing_read_each": (c_int, [c_void_p, _pd, c_int64, _pi64]),
    "mc_timing_read_spans": (c_int, [c_void_p, _pd, c_int64, _pi64]),
    "mc_set_launch": (c_int, [c_void_p, c_int32]),
    "mc_comm_unique_id": (c_int, [POINTER(c_char)]),
    "mc_comm_init": (c_int, [c_void_p, c_int, c_int, POINTER(c_char), POINTER(c_void_p)]),
    "mc_comm_destroy": (c_int, [c_void_p]),
    "mc_comm_gather_batch": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "mc_comm_allreduce_max_f64": (c_int, [c_void_p, _pd, c_int64]),
    "mc_gather_plan": (c_int, [c_int32, c_int32, _pi64, _pi64, c_int64, c_int32, _pi64, _pi64, _pi64]),
    "mc_gather_batches": (c_int, [c_void_p, c_int32, c_void_p, c_int32, c_void_p]),
}
EXPORTED = tuple(_SIGS)

_lib = None


def load(path: str | None = None):
    """Load (once) and return the ctypes handle; raises McLibraryError when unusable."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise McLibraryError(
            f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C livox-motion-compensation-sim_amd/csrc` (no CPU fallback exists)")
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:  # pragma: no cover - depends on the image
        raise McLibraryError(f"cannot load {p}: {e}") from e
    for name, (res, args) in _SIGS.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if path is None:   # the in-tree library must export every entry point
                raise
            continue           # an explicit older build (tools/ab*.py arms): its own entry points only
        fn.restype = res
        fn.argtypes = args
    if lib.mc_abi_version() != 1:
        raise McLibraryError("libmcdeskew ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str = "", lib=None) -> None:
    """Map a C status code to the reference-compatible Python exception."""
    if rc == MC_OK:
        return
    src = lib if lib is not None else _lib
    msg = (src.mc_last_error() or b"").decode(errors="replace") if src is not None else ""
    if what:
        msg = f"{what}: {msg}"
    if rc == MC_ERR_INVALID:
        raise ValueError(msg)
    if rc == MC_ERR_INDEX:
        raise IndexError(msg)
    if rc == MC_ERR_NOMEM:
        raise MemoryError(msg)
    raise McError(f"[{rc}] {msg}")


def ptr(a, ctype):
    """Pointer to the data of a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(POINTER(ctype))


def fptr(a, ctype):
    """ptr() for the per-call latency path: a ctype instance over a's buffer, which POINTER(ctype)
    argtypes pass by reference (~0.7 us instead of ~2.7 us for data_as); read-only or empty arrays
    take ptr()."""
    try:
        return ctype.from_buffer(a)
    except (TypeError, ValueError):
        return ptr(a, ctype)
