"""MI355X-native LiDAR motion compensation — the hot path of
manishborikar92/livox-motion-compensation-sim, rebuilt on hand-written gfx950 HIP kernels.

Import with ``importlib.import_module("livox-motion-compensation-sim_amd")`` (the directory
name carries hyphens) or via the repo-root helper ``mcamd.py``.

Drop-in surface (reference file:line in each docstring):
  LiDARMotionSimulator   lidar_motion_compensation.py:274-859 (config contract, pose tables,
                         transform_pointcloud, batched frame loop, merge)
  MotionCompensator      livox_mid70_complete_simulator.py:1426-1536 (+ driver 2086-2105)
  LiDARPoint, IMUData    livox_mid70_complete_simulator.py:97-129
  LivoxLVXWriter, codecs lidar_motion_compensation.py:24-272, 932-948 (byte-exact LVX / PCD)
  CoordinateTransformer  livox_mid70_complete_simulator.py:145-233, 2107-2180 (coords)
Device layer: Context, Batch (blocked-CSR float32 columns in HBM); multi-GPU: dist.
"""
from . import _lib, codecs, config, coords, dist, runtime, trajectory  # noqa: F401
from .coords import CoordinateSystem, CoordinateTransformer, GPSData  # noqa: F401
from .codecs import LivoxLVXWriter  # noqa: F401
from ._lib import McError, McLibraryError  # noqa: F401
from .compensator import IMUData, LiDARPoint, MotionCompensator, imu_to_arrays  # noqa: F401
from .config import default_config, validate_config  # noqa: F401
from .runtime import Batch, Context, default_context  # noqa: F401
from .simulator import LiDARMotionSimulator  # noqa: F401

__version__ = "0.1.0"
