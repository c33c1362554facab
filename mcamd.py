"""Importable alias of the ``livox-motion-compensation-sim_amd`` package (its directory name
carries hyphens, which the ``import`` statement cannot spell)."""
import importlib
import os
import sys

_ROOT = os.path.dirname(os.path.abspath(__file__))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

_pkg = importlib.import_module("livox-motion-compensation-sim_amd")
sys.modules[__name__] = _pkg
