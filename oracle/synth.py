"""Synthetic Mid-70 frame generator — numpy mirror of the device generator ``k_synth``.

TEST INFRASTRUCTURE ONLY (see oracle/restatement.py header): used by tests, smoke() and
bench.py's cpu_baseline leg to rebuild on the host the exact points the GPU generated.

The reference never produces 100k-point frames, so BASELINE configs need a
generator.  Counter-based (splitmix64 finaliser) so that any frame can be regenerated
independently and the numpy and HIP versions are bit-identical: integer hashing, then
uniforms u = (h >> 40) * 2^-24 (exact in f32), then float32 multiply/add with round-to-nearest
and no contraction.  Points lie inside the Mid-70 FOV (70.4 x 77.2 deg, CSIM:66-67):
x = depth in [0.05, 90) m, y = x*tan(az), z = x*tan(el); intensity U[0,1);
t_ns = i * 1e8 // n spreads the returns over the 0.1 s frame (100k pts/s, CSIM:79-80,
matching CSIM:1048's 1000 ns spacing at 100k points).
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
DEPTH_SCALE = np.float32(float.fromhex("0x1.67cccc0p+6"))   # 89.95
DEPTH_MIN = np.float32(float.fromhex("0x1.99999a0p-5"))     # 0.05
TAN_H = np.float32(float.fromhex("0x1.692d20p-1"))          # tan(35.2 deg)
TAN_V = np.float32(float.fromhex("0x1.98b968p-1"))          # tan(38.6 deg)


def mix64(z: np.ndarray) -> np.ndarray:
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def frame_key(seed: int, frame_seed: int) -> np.uint64:
    with np.errstate(over="ignore"):
        s = (np.uint64(seed % 2**64) + np.uint64(frame_seed % 2**64)) * GAMMA
    return mix64(np.array([s], dtype=np.uint64))[0]


def synth_frame(n: int, seed: int, frame_seed: int):
    """One frame: returns (x, y, z, intensity) float32 arrays and t_ns int32 (len n)."""
    key = frame_key(seed, frame_seed)
    i = np.arange(n, dtype=np.uint64)
    c = np.uint64(4) * i
    with np.errstate(over="ignore"):
        u = [(mix64(key + (c + np.uint64(j + 1)) * GAMMA) >> np.uint64(40)).astype(np.float32)
             * np.float32(2.0 ** -24) for j in range(4)]
    x = (u[0] * DEPTH_SCALE).astype(np.float32) + DEPTH_MIN
    ah = ((u[1] * np.float32(2.0)) - np.float32(1.0)) * TAN_H
    av = ((u[2] * np.float32(2.0)) - np.float32(1.0)) * TAN_V
    y = x * ah
    z = x * av
    t = ((np.arange(n, dtype=np.int64) * 100_000_000) // max(n, 1)).astype(np.int32)
    return x.astype(np.float32), y.astype(np.float32), z.astype(np.float32), u[3].astype(np.float32), t


def synth_batch(counts, seed: int = 0, frame_id_base: int = 1000):
    """Frames f = 0..F-1 with frame_seed = frame_id_base + f (== mc_batch_synth)."""
    cols = [synth_frame(int(n), seed, frame_id_base + f) for f, n in enumerate(counts)]
    if not cols:
        e = np.zeros(0, np.float32)
        return e, e, e, e, np.zeros(0, np.int32)
    return tuple(np.concatenate([c[j] for c in cols]) for j in range(5))
