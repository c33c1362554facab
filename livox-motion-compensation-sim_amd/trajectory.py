"""Pose-table producers — host-side numpy, input only.

These mirror the reference's generators so that a drop-in run reproduces the reference's pose
tables bit-for-bit (same numpy ops in the same order, same global RNG stream):
  generate_trajectory  LMC:361-407
  add_sensor_noise     LMC:409-428
  lidar_times          LMC:792-793
They produce at most a few thousand rows (<= 72 KB) and are uploaded once per run; the per-point
work happens on the GPU.  ``imu_from_trajectory`` builds a 200 Hz gyro stream shaped like CSIM's
IMUSimulator output (CSIM:1191-1240) for Path-B benches.
"""
from __future__ import annotations

import numpy as np


def generate_trajectory(config: dict) -> dict:
    """LMC:361-407.  Unknown trajectory_type raises UnboundLocalError like the reference (LMC:389)."""
    t = np.linspace(0, config["duration"], int(config["duration"] * config["gps_rate"]))
    kind = config["trajectory_type"]
    if kind == "linear":
        x = config["max_speed"] * t
        y = 5 * np.sin(0.1 * t)
        z = np.zeros_like(t)
    elif kind == "circular":
        radius = 50.0
        angular_freq = config["max_speed"] / radius
        x = radius * np.cos(angular_freq * t)
        y = radius * np.sin(angular_freq * t)
        z = np.zeros_like(t)
    elif kind == "figure_eight":
        scale = 30.0
        freq = 0.05
        x = scale * np.sin(2 * np.pi * freq * t)
        y = scale * np.sin(4 * np.pi * freq * t)
        z = np.zeros_like(t) + 1.5
    else:
        raise UnboundLocalError("cannot access local variable 'x' where it is not associated with a value")
    vx = np.gradient(x) * config["gps_rate"]
    vy = np.gradient(y) * config["gps_rate"]
    vz = np.gradient(z) * config["gps_rate"]
    yaw = np.arctan2(vy, vx)
    pitch = np.zeros_like(t)
    max_roll = np.radians(5)
    roll = max_roll * np.sin(0.5 * yaw) * (np.sqrt(vx ** 2 + vy ** 2) / config["max_speed"])
    return {
        "time": t,
        "position": np.column_stack([x, y, z]),
        "velocity": np.column_stack([vx, vy, vz]),
        "orientation": np.column_stack([roll, pitch, yaw]),
    }


def add_sensor_noise(trajectory: dict, config: dict) -> dict:
    """LMC:409-428 — draws from the global np.random stream (seeded at construction, LMC:288)."""
    gps_noise = np.random.normal(0, config["gps_noise_std"], trajectory["position"].shape)
    trajectory["position_gps"] = trajectory["position"] + gps_noise
    accel_noise = np.random.normal(0, config["imu_accel_noise"], trajectory["velocity"].shape)
    gyro_noise = np.random.normal(0, config["imu_gyro_noise"], trajectory["orientation"].shape)
    dt = 1.0 / config["gps_rate"]
    acceleration = np.gradient(trajectory["velocity"], dt, axis=0)
    trajectory["acceleration"] = acceleration + accel_noise
    trajectory["orientation_imu"] = trajectory["orientation"] + gyro_noise
    return trajectory


def lidar_times(config: dict) -> np.ndarray:
    """LMC:792-793 frame time grid (linspace, spacing duration/(n-1))."""
    return np.linspace(0, config["duration"], int(config["duration"] * config["lidar_fps"]))


def imu_from_trajectory(trajectory: dict, rate_hz: float = 200.0, duration: float | None = None):
    """200 Hz (timestamp_ns int64, gyro (M,3)) stream from a pose table, shaped like CSIM's
    IMUSimulator: int(t*1e9) timestamps (CSIM:1203), Euler-angle finite-difference gyro
    (CSIM:1210-1215; noise-free, zero first sample)."""
    t0 = trajectory["time"]
    if duration is None:
        duration = float(t0[-1])
    t = np.arange(0, duration, 1.0 / rate_hz)
    ori = np.stack([np.interp(t, t0, trajectory["orientation_imu"][:, j]) for j in range(3)], axis=1)
    gyro = np.zeros_like(ori)
    gyro[1:] = (ori[1:] - ori[:-1]) * rate_hz
    return (t * 1e9).astype(np.int64), gyro
