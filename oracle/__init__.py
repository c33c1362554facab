"""Parity oracle — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's motion-compensation path (restatement.py) and the numpy
mirror of the device's synthetic frame generator (synth.py).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this package, and only as the checker or the timed CPU
baseline; the product package never does.  Parity: pinned against golden vectors generated from
the reference itself (tests/golden/make_golden.py).
"""
from . import codecs, restatement, synth  # noqa: F401
