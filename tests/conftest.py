import importlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# parity tolerance (north_star: <= 1e-5 relative per coordinate).  Relative to the point's
# scale |p| + |t|: a floor-less per-coordinate relative error is meaningless on
# coordinates that cancel to ~0 after rotation.
REL_TOL = 1e-5


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU and the built libmcdeskew.so")


def pkg():
    return importlib.import_module("livox-motion-compensation-sim_amd")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def scale_of(points_xyz, translation=None):
    s = np.linalg.norm(np.asarray(points_xyz, dtype=np.float64), axis=-1)
    if translation is not None:
        t = np.asarray(translation, dtype=np.float64)
        s = s + (np.linalg.norm(t, axis=-1) if t.ndim > 1 else np.linalg.norm(t))
    return s


def assert_scaled_close(out, ref, scale, tol=REL_TOL, what=""):
    """max |out-ref| per coordinate <= tol * scale (per point); returns the worst ratio."""
    out = np.asarray(out, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert out.shape == ref.shape, f"{what}: shape {out.shape} != {ref.shape}"
    if out.size == 0:
        return 0.0
    err = np.abs(out - ref)
    if err.ndim == 2:
        err = err.max(axis=1)
    ratio = err / np.maximum(np.asarray(scale, dtype=np.float64), 1e-30)
    worst = float(ratio.max())
    assert worst <= tol, f"{what}: scaled error {worst:.3e} > {tol:.1e} at point {int(ratio.argmax())}"
    return worst


@pytest.fixture(scope="session")
def mc():
    return pkg()


@pytest.fixture(scope="session")
def gpu_ctx():
    m = pkg()
    try:
        n = m.Context.device_count()
    except Exception as e:  # the HIP path must exist on a GPU box: fail, never skip silently
        pytest.fail(f"libmcdeskew / HIP unusable: {e}")
    if n < 1:
        pytest.fail("no GPU visible to the HIP runtime")
    return m.Context(0)
