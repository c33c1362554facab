"""The bench line's contract at N > 1 (CPU; no GPU): what the driver's 8-GPU run will print.

SURVEY §8e asks for kernel scaling and the merged-cloud gather reported separately: ``value`` is the
timed steps' points over the max-over-ranks wall time (no gather inside), ``gather`` carries the
gather's own seconds / bytes into the root / GB/s, and the line holds its own 1-GPU denominator
(``single_gpu_same_job``) and ``speedup_vs_1gpu``; ``n_gpus`` counts distinct devices (bench.py
assemble_line, fed here with the values a sharded run produces)."""
import argparse
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


def _line(bench, world, n_devices, gather, single, mode="pose_slerp"):
    args = argparse.Namespace(mode=mode, warmup=5, issue="pipeline", events_after=False)
    counts_all = np.full(6000, 100_000, np.int64)
    bounds = bench.mc.dist.plan_shards(counts_all, world)
    lo, hi = int(bounds[0]), int(bounds[1])
    n_rank = int(counts_all[lo:hi].sum())
    n_total = int(counts_all.sum())
    steps, wall = 20, 20 * 400e-6
    kern_us = 330.0
    results = {mode: {"wall_s": wall, "steps": steps, "main_avg_us": kern_us, "timed_launches": 4,
                      "prep_avg_us": None, "achieved_GBs": 36 * n_rank / (kern_us * 1e-6) / 1e9,
                      "value": n_total * steps / wall / 1e6}}
    return bench.assemble_line(args, 4, bench.CONFIGS[4]["label"], "urban_complex", lo, hi, world, n_devices,
                               n_rank, n_total, counts_all, results, 250.0, 5, {}, None, None, None, None, gather,
                               False, single)


def test_n8_line_carries_kernel_value_gather_and_single_gpu_denominator(bench):
    gather = {"seconds": 0.42, "bytes_into_root": 16 * 525_000_000, "GBs": 20.0, "merged_points": 600_000_000,
              "timed_on": "root wall clock", "parity": {"ok": True}}
    single = {"value": 177_000.0, "unit": "Mpoints/s", "ms_per_step": 3.4, "kernel_avg_us": 3384.0,
              "frac": 0.8, "points": 600_000_000, "steps": 20}
    line = _line(bench, 8, 8, gather, single)
    assert line["n_gpus"] == 8
    assert line["config"]["ranks"] == 8 and line["config"]["devices"] == 8
    assert line["scaling"] == "strong"
    # value = kernels only: all ranks' points of the K timed steps / max wall, the gather excluded
    assert line["value"] == pytest.approx(600_000_000 * 20 / (20 * 400e-6) / 1e6)
    assert {"seconds", "bytes_into_root", "GBs"} <= set(line["gather"])
    assert line["gather_ok"] is True and line["ok"] is True
    assert line["single_gpu_same_job"] is single
    assert line["speedup_vs_1gpu"] == pytest.approx(line["value"] / single["value"])
    assert line["roofline"]["points_per_launch"] == 75_000_000   # the rank's shard (750 frames)
    assert line["roofline"]["frac"] == pytest.approx(line["roofline"]["achieved"] / 8000.0)


def test_shared_device_and_failed_gather_are_flagged(bench):
    line = _line(bench, 2, 1, {"error": "ncclCommInitRank: invalid usage"}, {"error": "skipped"})
    assert "NOT a scaling result" in line["scaling"]
    assert line["gather_ok"] is False and line["ok"] is False
    assert line["speedup_vs_1gpu"] is None
