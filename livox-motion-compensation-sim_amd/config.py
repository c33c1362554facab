"""The LiDARMotionSimulator config-dict contract (SURVEY §8b "Config"), kept verbatim.

default_config     LMC:297-330  (same keys, same defaults)
validate_config    LMC:332-359  (same checks, same ValueError messages, same order)
Merge order and seeding are applied by ``LiDARMotionSimulator.__init__`` exactly as LMC:282-288.
"""
from __future__ import annotations


def default_config() -> dict:
    """LMC:297-330."""
    return {
        # Simulation parameters
        "duration": 60.0,
        "lidar_fps": 10,
        "imu_rate": 100,
        "gps_rate": 5,
        "random_seed": 42,
        # Motion parameters
        "max_speed": 15.0,
        "max_angular_vel": 0.5,
        "trajectory_type": "figure_eight",
        # LiDAR Mid-70 specifications
        "fov_horizontal": 70.0,
        "fov_vertical": 77.2,
        "range_max": 90.0,
        "range_min": 0.05,
        "points_per_frame": 96000,
        "angular_resolution": 0.28,
        # Noise parameters
        "gps_noise_std": 0.03,
        "imu_accel_noise": 0.1,
        "imu_gyro_noise": 0.01,
        "lidar_range_noise": 0.02,
        # Environment parameters
        "environment_complexity": "medium",
        "ground_height": 0.0,
        "obstacle_density": 0.1,
    }


def validate_config(config: dict) -> None:
    """LMC:332-359: raises ValueError on invalid values (checks only the keys present)."""
    numeric_keys = ["duration", "lidar_fps", "max_speed", "range_max", "range_min", "points_per_frame"]
    for key in numeric_keys:
        if key in config and not isinstance(config[key], (int, float)):
            raise ValueError(f"Configuration '{key}' must be numeric")
    if "lidar_fps" in config and config["lidar_fps"] <= 0:
        raise ValueError("LiDAR frame rate must be positive")
    if "duration" in config and config["duration"] <= 0:
        raise ValueError("Simulation duration must be positive")
    if "max_speed" in config and config["max_speed"] < 0:
        raise ValueError("Maximum speed cannot be negative")
    if "range_max" in config and "range_min" in config:
        if config["range_max"] <= config["range_min"]:
            raise ValueError("Maximum range must be greater than minimum range")
