"""Benchmark: Mpoints/s deskewed + % of HBM roofline on synthetic Mid-70 frames, BASELINE configs.

One step = one pass of the hot path over the rank's batch: the per-step pose prep (pose selection /
segment tables, LMC:804-812) + the deskew kernel over every point of the rank's frames.  Inputs are
generated on the device and are resident in HBM before the timed region.

Workload = a BASELINE config (BASELINE.json "configs"), whose frames shard by index across the ranks
as contiguous point-balanced ranges (dist.plan_shards) — no collective on the data path:
    --config 2  urban_complex figure_eight, 600 frames x 100k        (default at 1 GPU)
    --config 3  parking_detailed circular, 600 x 100k, noise on
    --config 4  urban_complex figure_eight, 6000 x 100k (duration 600 s; 750 per GPU at 8)
                                                                      (default at N > 1 GPUs)
    --config 5  urban_complex poses, 1200 x 1M-point dense frames (150 per GPU at 8)
    --config 1  highway_simple linear, 10 x 20k (the reference's CPU case; launch-bound)
The total job is fixed per config ("scaling": "strong").  --frames F [--points n] instead runs F
frames per GPU of a longer run (weak scaling, the round-1 default).

After the timed steps (outside the timed region): the rank's output is spot-checked against the
oracle (N = 1), or, at N > 1, the merged cloud is gathered to rank 0 over RCCL (LMC:887-889), timed,
and sampled frames of every rank's shard are checked against the oracle (``gather.parity``).  A
failed or hung gather or a parity miss exits non-zero after the JSON line.

Beside the headline (same line, never part of ``value``): the other two modes, the stager pair,
scan_environment, the LVX / PCD writers after a fresh deskew and cold (``codecs``), and at N = 1 the
reference's host-array calling convention at config-2 scale (``host_path``: run_alignment on numpy
frames, against the box's PCIe DMA rates) and the simulate_frames -> save_results sequence
(``simulate_save``); the reference's op sequence on the box's cores (``cpu_baseline``).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode pose_slerp|frame|imu] [--config C]
    torchrun --nproc-per-node N ... bench.py --gpus N   (one process per GPU, RCCL over xGMI)

``python bench.py --gpus N`` (N > 1) without a torchrun environment launches the N rank processes
itself (launch_ranks: child processes, never exec; the parent loads no HIP library), forwards rank
0's line and fails if any rank fails.  At N > 1 rank 0 also times the same whole job on its own GPU
alone after the sharded run (``single_gpu_same_job``, ``speedup_vs_1gpu``).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import mcamd as mc  # noqa: E402

BYTES_PER_POINT = {"pose_slerp": 36, "imu": 36, "frame": 32}   # SURVEY §8d algorithmic bytes
HBM_PEAK_GBS = 8000.0                                          # MI355X_MICROARCH.md chip table
KERNEL = {"pose_slerp": "k_deskew_points<1", "imu": "k_deskew_points<2", "frame": "k_deskew_frame"}
# the kernel each issue mode times (pipeline: the step's deskew with the next step's prep in its first
# workgroups; the last step's launch is the plain kernel)
KERNEL_OF = {"pipeline": {"pose_slerp": "k_deskew_points<1, true, false>", "imu": "k_deskew_points<2, true, false>",
                          "frame": "k_deskew_frame_next"},
             "calls": {"pose_slerp": "k_deskew_points<1, false, false>", "imu": "k_deskew_points<2, false, false>",
                       "frame": "k_deskew_frame"}}
REL_TOL = 1e-5                                                 # north_star, relative per coordinate

SCENARIOS = {   # LMC:1182-1204
    "urban_complex": {"duration": 120.0, "trajectory_type": "figure_eight", "environment_complexity": "complex",
                      "max_speed": 12.0, "lidar_fps": 10},
    "parking_detailed": {"duration": 30.0, "trajectory_type": "circular", "environment_complexity": "medium",
                         "max_speed": 5.0, "lidar_fps": 20},
    "highway_simple": {"duration": 60.0, "trajectory_type": "linear", "environment_complexity": "simple",
                       "max_speed": 25.0, "lidar_fps": 15},
}
CONFIGS = {    # BASELINE.json "configs" (index = position + 1)
    1: {"scenario": "highway_simple", "frames": 10, "points": 20_000,
        "label": "BASELINE config 1: highway_simple linear, 10 frames x 20k pts"},
    2: {"scenario": "urban_complex", "frames": 600, "points": 100_000,
        "label": "BASELINE config 2: urban_complex figure_eight, 600 frames x 100k pts"},
    3: {"scenario": "parking_detailed", "frames": 600, "points": 100_000,
        "label": "BASELINE config 3: parking_detailed circular, 600 frames x 100k pts, IMU/GPS noise on"},
    4: {"scenario": "urban_complex", "frames": 6000, "points": 100_000, "duration": 600.0,
        "label": "BASELINE config 4: urban_complex figure_eight, 6000 frames x 100k pts sharded over the GPUs, "
                 "RCCL gather of merged_aligned"},
    5: {"scenario": "urban_complex", "frames": 1200, "points": 1_000_000,
        "label": "BASELINE config 5: 1200 x 1M-pt dense frames (urban_complex poses), HBM-roofline stress"},
}


def cpu_cores() -> dict:
    """Host cores this process may use: the affinity mask, bounded by a cgroup CPU quota if any."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, math.ceil(quota)))
    return {"affinity": aff, "cgroup_quota_cpus": quota, "usable": usable}


def workload(args, rank, world):
    """(config id or None, label, scenario cfg, pose table, global frame times, global counts,
    this rank's frame range [lo, hi))."""
    if args.frames is not None:      # custom weak-scaling job: args.frames per GPU
        cid, scen, F, n = None, args.scenario, args.frames * world, args.points
        base = SCENARIOS[scen]
        cfg = dict(base, duration=max(base["duration"], F / base["lidar_fps"]))
        label = f"custom: {scen}, {args.frames} frames x {n} pts per GPU (weak scaling)"
    else:
        cid = args.config if args.config != "auto" else (2 if world == 1 else 4)
        cid = int(cid)
        c = CONFIGS[cid]
        scen, F, n = c["scenario"], c["frames"], c["points"]
        cfg = dict(SCENARIOS[scen])
        if "duration" in c:
            cfg["duration"] = c["duration"]
        label = c["label"]
    sim = mc.LiDARMotionSimulator(cfg)       # seeds numpy's global RNG (LMC:288), seed 42
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:F]
    assert len(times) == F, (len(times), F)
    counts = np.full(F, n, dtype=np.int64)
    b = mc.dist.plan_shards(counts, world)
    return cid, label, scen, cfg, tr, times, counts, int(b[rank]), int(b[rank + 1])


# ---------------------------------------------------------------------------------------------
# oracle checks (outside the timed region)
# ---------------------------------------------------------------------------------------------
def oracle_frame(mode, tr, t_frame, start_ns, imu, n, frame_id):
    """The oracle's output for one synthetic frame (global frame id) and its per-point scale."""
    from oracle import restatement as R
    from oracle import synth
    x, y, z, i, t = synth.synth_frame(n, 0, 1000 + frame_id)
    p = np.stack([x, y, z], 1).astype(np.float64)
    if mode == "pose_slerp":
        ref = R.deskew_pose_slerp(p, t, t_frame, tr)
        _, pos = R.slerp_pose(tr["time"], tr["position_gps"], tr["orientation_imu"], t_frame + t * 1e-9)
        scale = np.linalg.norm(p, axis=1) + np.linalg.norm(pos, axis=1)
    elif mode == "frame":
        k = int(R.select_pose_index(tr["time"], t_frame))
        ref = p @ R.euler_xyz_matrix(tr["orientation_imu"][k]).T + tr["position_gps"][k]
        scale = np.linalg.norm(p, axis=1) + np.linalg.norm(tr["position_gps"][k])
    else:
        ref = R.compensate_arrays(p, start_ns + t.astype(np.int64), start_ns, imu[0], imu[1])
        scale = np.linalg.norm(p, axis=1)
    return ref, scale, i


def check_frames(batch, mode, tr, times, imu, counts, local_frames, global_ids):
    """Frames of ``batch`` (local indices) against the oracle (global frame ids): every coordinate
    within 1e-5 relative (north_star: |a-b| / |b|, |b| floored at 1e-9 * (|p|+|t|)), and the scaled
    error |a-b| / (|p|+|t|) beside it."""
    worst, naive = 0.0, []
    bad_int = 0
    for lf, gf in zip(local_frames, global_ids):
        got = batch.download_frames(lf, lf + 1)
        ref, scale, inten = oracle_frame(mode, tr, float(times[gf]), int(times[gf] * 1e9), imu, int(counts[gf]), gf)
        err = np.abs(got[:, :3] - ref)
        worst = max(worst, float((err.max(axis=1) / scale).max()) if len(ref) else 0.0)
        naive.append((err / np.maximum(np.abs(ref), 1e-9 * scale[:, None])).ravel())
        bad_int += int(np.count_nonzero(got[:, 3] != inten.astype(np.float64)))
    nv = np.concatenate(naive) if naive else np.zeros(0)
    above = int(np.count_nonzero(nv > REL_TOL))
    return {"frames_checked": [int(g) for g in global_ids], "worst_scaled_err": worst, "tol": REL_TOL,
            "ok": bool(worst <= REL_TOL and above == 0 and bad_int == 0), "intensity_mismatches": bad_int,
            "naive_rel_err": {"max": float(nv.max()) if nv.size else 0.0,
                              "p99_9": float(np.quantile(nv, 0.999)) if nv.size else 0.0,
                              "median": float(np.median(nv)) if nv.size else 0.0,
                              "coords_above_1e-5": above, "coords": int(nv.size),
                              "note": "the gate: |a-b|/|b| per coordinate <= 1e-5 (north_star), |b| floored at "
                                      "1e-9 * (|p|+|t|); float64 arithmetic in the kernels, one float32 rounding "
                                      "on the store"}}


# ---------------------------------------------------------------------------------------------
# CPU baseline (before the GPU is touched; the all-cores legs spawn worker processes)
# ---------------------------------------------------------------------------------------------
CPU_CACHE_FRAMES = 48   # synthetic frames a CPU worker generates once and then cycles through


def _cpu_frames(mode, tr, times, counts, frame_lo, budget_s, f_first=0, f_step=1, start_at=None):
    """The oracle on frames f_first, f_first+f_step, ... (cycling through them again while compute
    time remains) until budget_s of compute, one BLAS thread.  Returns (points, seconds, frames, late
    start s).  frame mode = the reference's own op sequence (scipy from_euler, R @ P.T, + t,
    column_stack; LMC:772-776) after the pose selection (804-812).  The worker's frames (at most
    CPU_CACHE_FRAMES) are generated before timing starts, so the budget is compute only (VERDICT r3:
    one pass over 600 frames gave a 16-process frame leg only 11-26 ms per worker).  Untimed first:
    one whole frame (imports scipy, faults in the buffers) — VERDICT r2: a fresh worker otherwise paid
    the cold scipy import inside its timed region.  ``start_at`` (wall clock): every worker of an
    all-cores leg starts timing at the same moment, so they run together."""
    from threadpoolctl import threadpool_limits
    from oracle import restatement as R
    from oracle import synth
    done = 0
    t_total = 0.0
    nf = 0
    ts_imu = gyro = None
    if mode == "imu":
        ts_imu, gyro = mc.trajectory.imu_from_trajectory(tr, 200.0)

    mine = list(range(f_first, len(counts), f_step))[:CPU_CACHE_FRAMES]
    cache = {}
    for f in mine:
        x, y, z, i, t = synth.synth_frame(int(counts[f]), 0, 1000 + frame_lo + f)
        cache[f] = (np.column_stack([x, y, z, i]).astype(np.float64), t)

    def one(f):
        pts, t = cache[f]
        t0 = time.perf_counter()
        if mode == "frame":
            k = int(R.select_pose_index(tr["time"], times[f]))
            R.transform_pointcloud_ref_ops(pts, {"translation": tr["position_gps"][k],
                                                 "rotation": tr["orientation_imu"][k]})
        elif mode == "pose_slerp":
            out = R.deskew_pose_slerp(pts[:, :3], t, times[f], tr)
            np.column_stack([out, pts[:, 3]])
        else:
            st = int(times[f] * 1e9)
            out = R.compensate_arrays(pts[:, :3], st + t.astype(np.int64), st, ts_imu, gyro)
            np.column_stack([out, pts[:, 3]])
        return time.perf_counter() - t0

    late = 0.0
    with threadpool_limits(limits=1):
        if mine:
            one(mine[0])                      # untimed warm-up frame
        if start_at is not None:
            wait = start_at - time.time()
            if wait > 0:
                time.sleep(wait)
            else:
                late = -wait
        k = 0
        while mine and t_total < budget_s:
            f = mine[k % len(mine)]
            t_total += one(f)
            done += int(counts[f])
            nf += 1
            k += 1
    return done, t_total, nf, late


def _cpu_worker(job):
    return _cpu_frames(*job)


def cpu_leg(mode, tr, times, counts, frame_lo, budget_s, procs, pool):
    n0 = int(counts[0]) if len(counts) else 0
    if procs <= 1:
        done, secs, nf, _ = _cpu_frames(mode, tr, times, counts, frame_lo, budget_s)
        return {"value": done / secs / 1e6, "unit": "Mpoints/s", "cores": 1, "blas_threads": 1,
                "compute_s": round(secs, 3),
                "sample": f"{nf} frame passes over {min(len(counts), CPU_CACHE_FRAMES)} of the {len(counts)} frames x "
                          f"{n0} pts, {secs:.1f} s of compute (after one untimed warm-up frame)"}
    start_at = time.time() + 10.0         # the workers are spawned and warmed up by then
    jobs = [(mode, tr, times, counts, frame_lo, budget_s, p, procs, start_at) for p in range(procs)]
    res = pool.map(_cpu_worker, jobs)
    pts = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    frames = sum(r[2] for r in res)
    return {"value": pts / wall / 1e6, "unit": "Mpoints/s", "cores": procs, "blas_threads": 1,
            "per_worker_compute_s": [round(r[1], 3) for r in res],
            "late_start_s": round(max(r[3] for r in res), 3),
            "sample": f"{frames} frame passes (frames x {n0} pts, round-robin over {procs} processes, each cycling "
                      f"through its frames for {budget_s:.1f} s of compute) after an untimed warm-up frame each, "
                      f"all starting at one wall-clock moment; rate = points / slowest worker's compute time"}


def cpu_baselines(mode, tr, times, counts, frame_lo, budget_s, procs):
    """The oracle on the same synthetic frames, generation excluded, each leg on one core and on
    ``procs`` processes (OPENBLAS threads = 1 everywhere).  The line's top-level value is the
    all-cores FRAME leg: the reference's own op sequence (LMC:772-776 — from_euler, R @ P.T, + t,
    column_stack per frame), the only CPU path the reference has for this hot path.
    The headline GPU mode's own oracle leg (SLERP: a build-added mode with no reference function)
    is reported beside it as ``legs[mode]``."""
    import multiprocessing as mp
    legs = ["frame"] + ([mode] if mode != "frame" else [])
    out = {}
    with mp.get_context("spawn").Pool(procs) if procs > 1 else _NullPool() as pool:
        for m in legs:
            single = cpu_leg(m, tr, times, counts, frame_lo, budget_s, 1, None)
            multi = cpu_leg(m, tr, times, counts, frame_lo, budget_s, procs, pool) if procs > 1 else None
            out[m] = {"single_core": single, "all_cores": multi}
            if multi is not None:
                out[m]["all_cores_ge_single"] = bool(multi["value"] >= single["value"])
                if multi["value"] < single["value"]:
                    print(f"warning: cpu baseline {m}: {procs} processes ({multi['value']:.1f} Mpoints/s) below one "
                          f"core ({single['value']:.1f})", file=sys.stderr)
    head = out["frame"]["all_cores"] or out["frame"]["single_core"]
    line = {"value": head["value"], "unit": "Mpoints/s", "cores": head["cores"], "kind": "port",
            "path": "reference op sequence (LMC:772-776, per frame after the LMC:804-812 pose selection)",
            "sample": "frame leg: " + head["sample"],
            "legs": out,
            "note": "oracle = numpy restatement of the reference's op sequence (oracle/restatement.py; "
                    "profiles/cpu_calibration.json: within 5 % of the reference's own transform_pointcloud), same "
                    "synthetic frames as the GPU, generation excluded; frame leg = scipy from_euler -> R @ P.T -> "
                    f"+ t -> column_stack per frame; legs[{mode!r}] = the headline GPU mode's oracle"}
    return line


class _NullPool:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


# ---------------------------------------------------------------------------------------------
# side measurements, unchanged contracts
# ---------------------------------------------------------------------------------------------
def traffic_file():
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)


def aux_traffic(*kernels):
    """PMC traffic / algorithmic bytes of the kernels around the path (tools/pmc_traffic.py --aux)."""
    d = traffic_file()
    got = {k: d[f"aux:{k}"]["traffic_over_algorithmic"] for k in kernels if f"aux:{k}" in d}
    return got or None


def load_traffic(mode, frames, points):
    """HBM bytes per launch of this mode at this per-GPU shape from profiles/pmc_traffic.json, with
    where it came from (a separate rocprofv3 --pmc session, not this run)."""
    e = traffic_file().get(f"{mode}:{frames}x{points}")
    if e is None:
        return None, None
    src = {"file": "profiles/pmc_traffic.json", "key": f"{mode}:{frames}x{points}", "session": e.get("tag"),
           "traffic_over_algorithmic": e.get("traffic_over_algorithmic"),
           "how": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes of bench.py (tools/pmc_traffic.py; "
                  "FETCH_SIZE x2 gfx950 correction), measured in that session, not in this run"}
    return e.get("hbm_bytes_per_launch"), src


def tune(ctx, mode, b_in, b_out):
    """Untimed, between the two halves of the spin-up (at sustained clocks): the device picks the
    mode's sub-tile order (dealt over the XCDs or XCD-contiguous, Context.tune_order /
    mc_tune_order): which one streams faster differs between kernels, store policies and MI355X
    boxes by up to 7 % for the same kernel."""
    return ctx.tune_order(b_in, b_out, mode=mode, launches=8, rounds=6)


def spin_up(ctx, mode, b_in, b_out, ms, issue):
    """Untimed: run the step itself for at least ``ms`` milliseconds before the warmup steps.  From
    idle the device takes tens of milliseconds of sustained load to reach its steady memory
    throughput — far longer than a few warmup steps (0.33 ms each): SLERP kernel 80.4-81.2 % of
    peak after 5 warmup steps, 84.1 % after 50, 84.6-84.8 % after 300, same box and buffers
    (profiles/round2/s51).  Returns the milliseconds spent."""
    if ms <= 0:
        return 0.0
    ctx.timing(False)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        if issue == "pipeline":
            ctx.deskew_steps(b_in, b_out, 25, mode=mode, sample_every=0)
        else:
            for _ in range(25):
                ctx.deskew(b_in, b_out, mode=mode)
        ctx.sync()
    return (time.perf_counter() - t0) * 1e3


def run_mode(ctx, rdv, mode, b_in, b_out, steps, warmup, live=True, issue="pipeline"):
    """Timed region: wall clock around ``steps`` steps.  ``live``: HIP events on the sampled steps'
    kernels themselves (hipExtLaunchKernel start/stop events: the dispatch's own timestamps, no
    marker packets between the steps) give the roofline's per-launch kernel time.  Otherwise a
    second, untimed pass carries events on every launch.  ``issue``: "pipeline" = one
    Context.deskew_steps call, each step's launch also running the next step's prep (the first
    step's prep is its own launch, inside the timed region); "calls" = ``steps`` Context.deskew
    calls (prep + kernel each)."""
    every = 10 if steps >= 50 else 5
    ctx.timing(live)           # warmup steps fill the context's event pool for the sampled steps
    for _ in range(warmup):
        ctx.deskew(b_in, b_out, mode=mode)
    if issue == "pipeline" and warmup:
        ctx.deskew_steps(b_in, b_out, warmup, mode=mode, sample_every=1 if live else 0)
    ctx.sync()
    ctx.timing(False)
    ctx.read_timing()          # drop the warmup events (back to the pool)
    rdv.barrier()
    t0 = time.perf_counter()
    if issue == "pipeline":
        ctx.deskew_steps(b_in, b_out, steps, mode=mode, sample_every=every if live else 0)
    else:
        for i in range(steps):
            sample = live and i % every == every // 2
            if sample:
                ctx.timing(True)
            ctx.deskew(b_in, b_out, mode=mode)
            if sample:
                ctx.timing(False)
    ctx.sync()
    t1 = time.perf_counter()
    rdv.barrier()
    if not live:
        if issue == "pipeline":
            ctx.deskew_steps(b_in, b_out, min(steps, 50), mode=mode, sample_every=1)
        else:
            ctx.timing(True)
            for _ in range(min(steps, 50)):
                ctx.deskew(b_in, b_out, mode=mode)
            ctx.timing(False)
        ctx.sync()
    each = ctx.read_timing_each()
    # the warmup launches' spans come first (reading them before the timed steps would idle the
    # device between warmup and timing: after ~1 ms idle the next tens of launches run through a
    # power transient, 317 -> 375 us, profiles/round4/s13 kernel trace)
    spans = ctx.read_timing_spans()[-len(each):] if each else []
    tm = ctx.read_timing()
    tm["main_ms"], tm["main_launches"], tm["main_each_us"] = sum(each), len(each), [round(x * 1e3, 2) for x in each]
    # the same launches' own execution spans (first workgroup start to last workgroup end): the
    # kernel time rocprofv3's kernel trace reports; the events also hold the dispatch gap ahead of
    # each launch (~5 us, profiles/round4/s12/roofline_trace.json)
    tm["main_span_us"] = [round(x, 2) for x in spans] if len(spans) == len(each) else None
    return t1 - t0, tm, every


def measure_stager(ctx, b_in, b_out, n_rank, reps):
    """SURVEY §8f row 1, reported beside the hot path: the device stager pair converting the
    reference's (N,4) float64 AoS to/from the float32 SoA columns, 48 algorithmic B/point."""
    buf = ctx.device_buffer(n_rank * 32)
    try:
        out = {}
        for name, fn in (("soa_to_aos", lambda: b_in.fetch_aos_device(buf)),
                         ("aos_to_soa", lambda: b_out.stage_aos_device(buf))):
            for _ in range(3):
                fn()
            ctx.sync()
            ctx.read_timing()
            ctx.timing(True)
            for _ in range(reps):
                fn()
            ctx.sync()
            ctx.timing(False)
            t = ctx.read_timing()
            us = t["layout_ms"] / max(t["layout_launches"], 1) * 1e3
            gbs = 48 * n_rank / (us * 1e-6) / 1e9
            out[name] = {"kernel_avg_us": us, "GBs": gbs, "frac": gbs / HBM_PEAK_GBS, "bytes_per_point": 48,
                         "traffic_over_algorithmic": aux_traffic("k_" + name)}
        return out
    finally:
        buf.close()


def measure_scan(ctx, cfg, tr, reps, cpu_budget):
    """SURVEY §8f row 2, reported beside the hot path: scan_environment for every frame of the
    urban_complex run (1200 frames, LMC:792-815) against a scene the size of the reference's urban
    scene (29,000 points, LMC:430-699), noise on.  Unit: scene points tested per second (F x E)."""
    rng = np.random.default_rng(7)
    E = 29_000
    env = np.column_stack([rng.uniform(-200, 200, E), rng.uniform(-200, 200, E), rng.uniform(-25, 70, E),
                           rng.uniform(0, 1, E)])
    urban = SCENARIOS["urban_complex"]
    times = mc.trajectory.lidar_times(dict(cfg, **urban))[:1200]
    F = len(times)
    scfg = dict(mc.default_config(), **urban)
    ctx.set_environment(env)
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    out = ctx.scan(times, scfg)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = ctx.scan(times, scfg, out=out)
    wall = (time.perf_counter() - t0) / reps
    ctx.read_timing()
    ctx.timing(True)
    for _ in range(reps):
        out = ctx.scan(times, scfg, out=out)
    ctx.timing(False)
    tm = ctx.read_timing()
    kern = tm["scan_ms"] / max(tm["scan_launches"], 1) * 2 / 1e3    # count + emit per scan
    rep = {"workload": f"{F} frames x {E} scene pts (urban_complex run, synthetic scene)",
           "wall_ms": wall * 1e3, "kernels_ms": kern * 1e3, "Mtests_s_wall": F * E / wall / 1e6,
           "Mtests_s_kernels": F * E / kern / 1e6, "points_out": int(out.n_points),
           "note": "wall includes host noise draw (numpy normal) + H2D of the noise"}
    if cpu_budget > 0:
        from oracle import restatement as R
        idx = R.select_pose_index(tr["time"], times)
        t_cpu, f = 0.0, 0
        while f < F and t_cpu < cpu_budget:
            pose = {"position": tr["position_gps"][idx[f]], "orientation": tr["orientation_imu"][idx[f]]}
            t1 = time.perf_counter()
            R.scan_environment(env, pose, scfg)
            t_cpu += time.perf_counter() - t1
            f += 1
        rep["cpu_baseline"] = {"Mtests_s": f * E / t_cpu / 1e6, "cores": 1, "kind": "port",
                               "sample": f"{f} frames, oracle numpy restatement"}
    return rep


def steady(ctx, fn, ms=100.0):
    """Untimed calls of fn for ~ms milliseconds before a measurement: these figures follow idle stretches
    of the bench (its CPU legs), and from idle the device needs tens of ms of load to reach its steady
    rate (as the headline's spin-up, spin_up)."""
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        fn()
        ctx.sync()


FLUSH_BYTES = 1 << 30   # cold runs: an untimed 512 MB -> 512 MB copy first (the Infinity Cache is 256 MB)


def measure_codecs(ctx, b_src, mode, b_out, n_rank, reps, cpu_budget):
    """SURVEY §8f row 3, reported beside the hot path: the byte-exact writers (LVX v1.1 LMC:24-272,
    ASCII PCD LMC:932-948) encoding the rank's whole deskewed batch straight from its float32
    columns in HBM (mc_*_encode_batch), timed the way the product runs them: every encode follows a
    fresh deskew of the batch (the reference's LMC:831 -> 887-889 -> 932-948 order), once
      after_deskew  directly (whatever of the batch the deskew left in the Infinity Cache is there)
      cold          after an untimed 512 MB -> 512 MB copy of unrelated data (none of it is)
    Kernel time only (HIP events of the encode's launches, median over reps); HBM bytes = 16 B/pt
    read + the encoded bytes written.  PCD: into a MC_BATCH_WITH_PCD_LEN batch the deskew kernel
    also writes each block's text length, so the encoder runs its write pass only; that pass + what
    the sums add to the deskew kernel (its median with sums minus without) is the PCD cost.  The
    two-pass encoder (measure + write) on a plain batch is reported beside it, the two interleaved
    rep by rep (so both deskews run unspeculated, in the same device state).  ``frac`` is the cold
    figure."""
    from ctypes import c_int64, c_uint64, c_void_p
    counts = np.ascontiguousarray(b_out.counts, np.int64)
    F = len(counts)
    ptr, check = mc._lib.ptr, mc._lib.check
    b_pcd = ctx.batch(counts, with_pcd_len=True)
    flush = ctx.device_buffer(FLUSH_BYTES)
    half = FLUSH_BYTES // 2
    hi = c_void_p(flush.ptr.value + half)

    def cold():
        check(ctx.lib.mc_memcpy_d2d(ctx.handle, hi, flush.ptr, half), "flush")

    def one(dst, encode, flushed):
        """flush -> deskew -> [flush] -> encode; the encode's kernel ms and the deskew's (main) kernel
        ms.  The first flush puts every deskew on the same footing (whatever encode ran before it),
        so the two PCD arms' deskews compare fairly."""
        cold()
        ctx.read_timing()
        ctx.timing(True)
        ctx.deskew(b_src, dst, mode=mode)
        ctx.timing(False)
        if flushed:
            cold()
        ctx.sync()
        ctx.timing(True)
        encode()
        ctx.timing(False)
        t = ctx.read_timing()
        return t["codec_ms"], t["main_ms"]

    def series(arms):
        """arms: name -> (deskew target, encode); the arms interleaved rep by rep, so every arm sees
        the same device state (and consecutive deskews into different batches: none is speculated)"""
        steady(ctx, lambda: [one(dst, enc, False) for dst, enc in arms.values()])
        res = {a: {"after_deskew": [], "cold": []} for a in arms}
        for _ in range(reps):
            for kind in ("after_deskew", "cold"):
                for a, (dst, enc) in arms.items():
                    res[a][kind].append(one(dst, enc, kind == "cold"))
        return {a: {k: (float(np.median([x for x, _ in v])), float(np.median([y for _, y in v])))
                    for k, v in r.items()} for a, r in res.items()}

    def figures(ms, alg):
        return {"kernels_ms": ms, "Mpoints_s": n_rank / ms / 1e3, "GBs": alg / ms / 1e6,
                "frac": alg / ms / 1e6 / HBM_PEAK_GBS}

    rep = {}
    pos = mc.codecs.lvx_layout(counts)
    ids = np.arange(F, dtype=np.uint64)
    ts = (np.arange(F) * 100_000_000).astype(np.uint64)
    out = ctx.device_buffer(int(pos[-1]))
    try:
        def lvx():
            check(ctx.lib.mc_lvx_encode_batch(ctx.handle, b_out.handle, ptr(ids, c_uint64), ptr(ts, c_uint64),
                                              out.ptr, int(pos[-1])), "lvx_encode_batch")
        m = series({"lvx": (b_out, lvx)})["lvx"]
    finally:
        out.close()
    alg = 16 * n_rank + int(pos[-1])
    rep["lvx"] = {"file_bytes": int(pos[-1]), "bytes_per_point": alg / n_rank,
                  "after_deskew": figures(m["after_deskew"][0], alg), "cold": figures(m["cold"][0], alg),
                  "traffic_over_algorithmic": aux_traffic("k_lvx_packages"),
                  "note": "each encode follows a fresh deskew of the batch; cold: after an untimed 512 MB copy"}
    rep["lvx"]["frac"] = rep["lvx"]["cold"]["frac"]

    bpos = np.zeros(F + 1, np.int64)
    cap = n_rank * 52
    text = ctx.device_buffer(cap)
    try:
        def pcd_into(b):
            def enc():
                check(ctx.lib.mc_pcd_encode_batch(ctx.handle, b.handle, text.ptr, cap, ptr(bpos, c_int64)),
                      "pcd_encode_batch")
            return enc
        m = series({"sum": (b_pcd, pcd_into(b_pcd)), "two": (b_out, pcd_into(b_out))})
        if not b_pcd.pcd_len_current():
            raise RuntimeError("the deskew into a MC_BATCH_WITH_PCD_LEN batch left no current text sums")
        m_sum, m_two = m["sum"], m["two"]
    finally:
        text.close()
        flush.close()
        b_pcd.close()
    tb = int(bpos[-1])
    alg = 16 * n_rank + tb
    sums_ms = {k: max(m_sum[k][1] - m_two[k][1], 0.0) for k in m_sum}
    rep["pcd_ascii"] = {"text_bytes": tb, "bytes_per_point": alg / n_rank,
                        "after_deskew": dict(figures(m_sum["after_deskew"][0] + sums_ms["after_deskew"], alg),
                                             write_ms=m_sum["after_deskew"][0],
                                             sums_in_deskew_us=sums_ms["after_deskew"] * 1e3),
                        "cold": dict(figures(m_sum["cold"][0] + sums_ms["cold"], alg), write_ms=m_sum["cold"][0],
                                     sums_in_deskew_us=sums_ms["cold"] * 1e3),
                        "two_pass": {"after_deskew": figures(m_two["after_deskew"][0], alg),
                                     "cold": figures(m_two["cold"][0], alg),
                                     "note": "plain batch: measure pass + write pass"},
                        "traffic_over_algorithmic": aux_traffic("k_pcd_write", "k_pcd_measure"),
                        "note": "MC_BATCH_WITH_PCD_LEN batch: the deskew writes the text sums, the encoder its "
                                "write pass only; cost = write pass + (deskew kernel with sums - without)"}
    rep["pcd_ascii"]["frac"] = rep["pcd_ascii"]["cold"]["frac"]
    if cpu_budget > 0:
        from oracle import codecs as C
        host = b_out.download_frames(0, 1)
        t0 = time.perf_counter()
        C.lvx_bytes([{"frame_id": 0, "timestamp": 0.0, "points": host}])
        t1 = time.perf_counter()
        k = min(len(host), 20_000)
        C.pcd_ascii_bytes(host[:k])
        t2 = time.perf_counter()
        rep["cpu_baseline"] = {"lvx_Mpoints_s": len(host) / (t1 - t0) / 1e6,
                               "pcd_Mpoints_s": k / (t2 - t1) / 1e6, "cores": 1, "kind": "port",
                               "sample": f"LVX 1 frame x {len(host)} pts (vectorised numpy oracle), "
                                         f"PCD {k} pts (Python float formatting, as the reference)"}
    return rep


def pcie_ceiling(nbytes=256 << 20, reps=5):
    """Pinned DMA rates of this box (HIP runtime through ctypes; tools/pcie_probe.py): H2D, D2H, and
    both at once on two streams (the aggregate the two directions carry together)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    bufs = [ctypes.c_void_p() for _ in range(4)]     # pinned, device, pinned, device
    out = {}
    streams = [ctypes.c_void_p(), ctypes.c_void_p()]
    try:
        for i, b in enumerate(bufs):
            rc = hip.hipHostMalloc(ctypes.byref(b), ctypes.c_size_t(nbytes), 0) if i % 2 == 0 else \
                hip.hipMalloc(ctypes.byref(b), ctypes.c_size_t(nbytes))
            if rc:
                raise RuntimeError("pcie_ceiling: allocation failed")
        pin, dev, pin2, dev2 = bufs
        for name, dst, src, kind in (("H2D", dev, pin, 1), ("D2H", pin, dev, 2)):
            hip.hipMemcpy(dst, src, ctypes.c_size_t(nbytes), kind)
            t0 = time.perf_counter()
            for _ in range(reps):
                hip.hipMemcpy(dst, src, ctypes.c_size_t(nbytes), kind)
            out[name + "_GBs"] = reps * nbytes / (time.perf_counter() - t0) / 1e9
        for st in streams:
            hip.hipStreamCreate(ctypes.byref(st))
        best = 0.0
        for _ in range(reps + 1):
            t0 = time.perf_counter()
            hip.hipMemcpyAsync(dev, pin, ctypes.c_size_t(nbytes), 1, streams[0])
            hip.hipMemcpyAsync(pin2, dev2, ctypes.c_size_t(nbytes), 2, streams[1])
            hip.hipStreamSynchronize(streams[0])
            hip.hipStreamSynchronize(streams[1])
            best = max(best, 2 * nbytes / (time.perf_counter() - t0) / 1e9)
        out["both_directions_GBs"] = best
    finally:
        for st in streams:
            if st.value:
                hip.hipStreamDestroy(st)
        for i, b in enumerate(bufs):
            if b.value:
                (hip.hipHostFree if i % 2 == 0 else hip.hipFree)(b)
    return out


def measure_host_path(ctx, cfg, frames, points, reps):
    """The reference's own calling convention at the workload's scale (BASELINE config 2: 600 x 100k;
    SURVEY §8 a3-a5 on host arrays): run_alignment on ``frames`` x ``points`` float64 (n, 4) numpy
    frames with the workload's scenario (``cfg``) poses, LMC:802-832, one
    call for all frames, host arrays in and out (the reference's transform_pointcloud returns a new
    array per frame: every call writes a fresh output, whose first-touch page faults are part of the
    wall time).  64 algorithmic bytes per point cross PCIe (32 in, 32 out); the ceilings are this
    box's pinned DMA rates: serial = one direction after the other (32/H2D + 32/D2H per point),
    concurrent = both directions at once as this box carries them (its measured aggregate / 64 B)."""
    rng = np.random.default_rng(0)
    base = rng.standard_normal((points, 4)) * 30.0
    scans = [base + f * 1e-3 for f in range(frames)]
    sim = mc.LiDARMotionSimulator(dict(cfg), context=ctx)
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()[:frames]
    sim.run_alignment(scans[:2], tr, times[:2])
    walls = []
    res = None
    for _ in range(reps):
        res = None
        t0 = time.perf_counter()
        res = sim.run_alignment(scans, tr, times)
        walls.append(time.perf_counter() - t0)
    # spot check, bit for bit, against the reference's op sequence (scipy R, numpy matmul) on two frames
    from oracle import restatement as R
    idx = R.select_pose_index(tr["time"], times)
    ok = True
    for f in (0, frames - 1):
        want = R.transform_pointcloud_ref_ops(scans[f], {"translation": tr["position_gps"][idx[f]],
                                                         "rotation": tr["orientation_imu"][idx[f]]})
        ok = ok and bool(np.array_equal(res[f], want))
    res = None
    pc = pcie_ceiling()
    n = frames * points
    best, med = min(walls), float(np.median(walls))
    serial = 1.0 / (32 / pc["H2D_GBs"] + 32 / pc["D2H_GBs"]) * 1e3          # Mpoints/s
    concurrent = pc["both_directions_GBs"] / 64 * 1e3
    return {"workload": f"run_alignment, {frames} x {points} float64 (n, 4) host frames (the bench workload's shape)",
            "wall_s": walls, "Mpoints_s": n / best / 1e6, "Mpoints_s_median": n / med / 1e6,
            "GBs_64B_per_point": 64 * n / best / 1e9, "pcie": pc,
            "ceiling_Mpoints_s": {"serial": serial, "concurrent": concurrent},
            "frac_pcie": n / best / 1e6 / serial, "frac_pcie_concurrent": n / best / 1e6 / concurrent,
            "bitwise_vs_reference_ops": ok,
            "note": "wall time of the drop-in call incl. its new output array (the first call; later ones reuse "
                    "a recycled block); frac_pcie against the serial ceiling (32 B/pt H2D then 32 B/pt D2H), "
                    "frac_pcie_concurrent against both directions at once as measured (two streams)"}


def measure_save(ctx, reps=1):
    """The reference's end-to-end sequence on the GPU drop-in: simulate_frames (LMC:802-858: every
    frame's scan + alignment, mc_scan_emit_f64) then save_results (LMC:860-931: CSVs, 2 x 1200
    per-frame PCDs, merged PCDs, LVX) for the urban_complex run over a synthetic scene the size of the
    reference's (29,000 points), written to a temporary directory.  The CPU figure is an estimate:
    the reference's per-line Python formatting (oracle.codecs.pcd_ascii_bytes, as LMC:946-948) timed
    on a sample of lines and scaled to the run's lines."""
    import shutil
    import tempfile
    rng = np.random.default_rng(7)
    E = 29_000
    env = np.column_stack([rng.uniform(-200, 200, E), rng.uniform(-200, 200, E), rng.uniform(-25, 70, E),
                           rng.uniform(0, 1, E)])
    sim = mc.LiDARMotionSimulator(dict(SCENARIOS["urban_complex"]), context=ctx)
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    d = tempfile.mkdtemp(prefix="mc_save_")
    import contextlib
    import io
    try:
        t0 = time.perf_counter()
        res = sim.simulate_frames(env, tr)
        t1 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            sim.save_results(res, d)
        t2 = time.perf_counter()
        files, nbytes = 0, 0
        for root, _, fs in os.walk(d):
            for fn in fs:
                files += 1
                nbytes += os.path.getsize(os.path.join(root, fn))
    finally:
        shutil.rmtree(d, ignore_errors=True)
    pts = sum(len(a) for a in res["aligned_pointclouds"])
    lines = 4 * pts      # raw + aligned per frame, and the two merged files
    from oracle import codecs as C
    sample = np.vstack(res["aligned_pointclouds"])[:20_000]
    t3 = time.perf_counter()
    C.pcd_ascii_bytes(sample)
    per_line = (time.perf_counter() - t3) / max(len(sample), 1)
    return {"workload": f"urban_complex run: {len(res['raw_scans'])} frames, {pts} points, synthetic 29k-point scene",
            "simulate_frames_s": t1 - t0, "save_results_s": t2 - t1, "total_s": t2 - t0,
            "files": files, "bytes": nbytes, "device_rows_reused": True,
            "cpu_estimate": {"pcd_lines_s": per_line * lines, "lines": lines, "cores": 1, "kind": "port",
                             "sample": f"{len(sample)} lines through the reference's per-line formatting"}}


def measure_deskew_pcd(ctx, b_in, b_out, mode, n_rank, reps):
    """SURVEY §8f row 3 fused with the path, both pipelines on the same batch, interleaved:
      separate  mc_deskew, then mc_pcd_encode_batch (measure pass + write pass)
      fused     mc_deskew_pcd: the deskew kernel also sums each 256-point block's ASCII PCD text
                bytes, then the write pass alone
    The fused PCD's cost is the write pass plus what the sums add to the deskew kernel (fused kernel
    minus the separate pipeline's plain kernel)."""
    from ctypes import c_int64
    counts = np.ascontiguousarray(b_out.counts, np.int64)
    pos = np.zeros(len(counts) + 1, np.int64)
    cap = int(counts.sum()) * 48
    buf = ctx.device_buffer(cap)
    ptr = mc._lib.ptr
    arms = {"separate": [], "fused": []}
    try:
        def separate():
            ctx.deskew(b_in, b_out, mode=mode)
            mc._lib.check(ctx.lib.mc_pcd_encode_batch(ctx.handle, b_out.handle, buf.ptr, cap, ptr(pos, c_int64)),
                          "pcd_encode_batch")

        def fused():
            mc._lib.check(ctx.lib.mc_deskew_pcd(ctx.handle, b_in.handle, b_out.handle, mc._lib.MODES[mode],
                                                mc._lib.POSE_SELECT["searchsorted"], buf.ptr, cap, ptr(pos, c_int64)),
                          "deskew_pcd")
        steady(ctx, lambda: (separate(), fused()))
        ctx.read_timing()
        for _ in range(reps):
            for name, fn in (("separate", separate), ("fused", fused)):
                ctx.timing(True)
                fn()
                ctx.timing(False)
                arms[name].append(ctx.read_timing())
    finally:
        buf.close()

    def med(name, key):   # median over the calls of the milliseconds the call's kernels of that kind took
        return float(np.median([t[key + "_ms"] for t in arms[name]]))
    k_sep, k_fus = med("separate", "main"), med("fused", "main")
    c_sep, c_fus = med("separate", "codec"), med("fused", "codec")
    text_b = int(pos[-1])
    alg = 16 * n_rank + text_b
    pcd_fused_ms = c_fus + max(k_fus - k_sep, 0.0)
    return {"mode": mode, "reps": reps, "text_bytes": text_b,
            "separate": {"deskew_kernel_us": k_sep * 1e3, "pcd_kernels_ms": c_sep, "total_ms": k_sep + c_sep},
            "fused": {"deskew_pcd_kernel_us": k_fus * 1e3, "write_ms": c_fus, "total_ms": k_fus + c_fus},
            "pcd_ms": pcd_fused_ms, "GBs": alg / pcd_fused_ms / 1e6, "frac": alg / pcd_fused_ms / 1e6 / HBM_PEAK_GBS,
            "frac_separate": alg / c_sep / 1e6 / HBM_PEAK_GBS,
            "note": "fused PCD cost = write pass + (deskew_pcd kernel - plain deskew kernel), medians over interleaved "
                    "calls; HBM bytes = 16 B/pt read + the text written (as codecs.pcd_ascii)"}


# ---------------------------------------------------------------------------------------------
# the merged-cloud gather (N > 1)
# ---------------------------------------------------------------------------------------------
def timed_gather(ctx, rdv, b_in, b_out, mode, n_rank, world, timeout_s, check):
    """The merged-cloud gather to rank 0 (LMC:887-889 over RCCL), after and outside the timed
    steps, under a watchdog.  ``check(merged)`` runs on the root afterwards (the parity of sampled
    frames).  Returns (report, hung).  The root's wall time is the gather time."""
    import threading
    res = {}

    def work():
        try:
            comm = mc.dist.RcclComm(ctx, rdv)
            ctx.deskew(b_in, b_out, mode=mode)
            ctx.sync()
            sizes = rdv.allgather(int(b_out.n_points))
            rdv.barrier()
            t0 = time.perf_counter()
            merged = mc.dist.gather_merged(ctx, comm, rdv, b_out, root=0)
            dt = time.perf_counter() - t0
            moved = 16 * (sum(sizes) - sizes[0])
            rep = {"seconds": dt, "bytes_into_root": moved, "GBs": moved / dt / 1e9,
                   "merged_points": int(sum(sizes)), "timed_on": "root wall clock"}
            if merged is not None:
                rep["parity"] = check(merged)
                merged.close()
            res["report"] = rep
            comm.close()
        except Exception as e:  # reported; the process exits non-zero after the line
            res["report"] = {"error": f"{type(e).__name__}: {e}"}

    th = threading.Thread(target=work, daemon=True)
    th.start()
    th.join(timeout_s)
    if th.is_alive():
        return {"error": f"gather did not finish within {timeout_s} s"}, True
    return res.get("report"), False


# ---------------------------------------------------------------------------------------------
# self-launch of the rank processes (python bench.py --gpus N, no torchrun environment)
# ---------------------------------------------------------------------------------------------
def _free_port_pair() -> int:
    """A MASTER_PORT whose +1 (the control plane's port, dist.Rendezvous) is free right now."""
    for _ in range(64):
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            s.bind(("127.0.0.1", 0))
            p = s.getsockname()[1]
        if p > 1024:
            return p - 1
    raise RuntimeError("no free port")


def launch_ranks(n: int, argv: list, timeout_s: float) -> int:
    """One child process per GPU with torch.distributed.run's environment (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT).  This process only waits: it never loads
    libmcdeskew or touches HIP, and starts the ranks as children (no exec).  Rank 0's stdout is
    forwarded; the exit code is the first failing rank's (a rank that fails makes the others stop
    within a grace period), 124 when the job runs past ``timeout_s`` (every rank killed)."""
    port = _free_port_pair()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MCBENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL, start_new_session=True))
    deadline = time.time() + timeout_s
    failed_at = None
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad and failed_at is None:
            failed_at = time.time()
            rc = bad[0]
        if all(c is not None for c in codes):
            break
        late = failed_at is not None and time.time() - failed_at > 60.0
        if time.time() > deadline or late:
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
            for p in procs:
                p.wait()
            print(f"bench launcher: {'timeout' if not late else 'a rank failed'}; ranks killed", file=sys.stderr)
            return rc or 124
        time.sleep(0.2)
    for r, p in enumerate(procs):
        if p.returncode != 0:
            print(f"bench launcher: rank {r} exited {p.returncode}", file=sys.stderr)
            return rc or p.returncode
    return 0


def control_plane_only(args) -> int:
    """--control-plane-only: the ranks rendezvous, exchange (rank, pid, host), take a max over
    ranks and a barrier — the multi-rank bookkeeping of the bench without a GPU.  Rank 0 prints one
    JSON line."""
    rank, local_rank, world = mc.dist.env_rank()
    # test hooks (tests/test_dist.py): one rank fails before the rendezvous, or hangs in it
    if os.environ.get("MCBENCH_FAIL_RANK") == str(rank):
        return 3
    if os.environ.get("MCBENCH_HANG_RANK") == str(rank):
        time.sleep(3600)
    rdv = mc.dist.Rendezvous(rank, world, timeout=float(os.environ.get("MCBENCH_RDV_TIMEOUT", "300")))
    info = rdv.allgather({"rank": rank, "local_rank": local_rank, "pid": os.getpid(), "host": socket.gethostname()})
    m = rdv.max(float(rank))
    rdv.barrier()
    if rank == 0:
        print(json.dumps({"control_plane": "ok", "world": world, "ranks": info, "max_over_ranks": m,
                          "launched_by": "bench.py" if os.environ.get("MCBENCH_LAUNCHED") else "external"}),
              flush=True)
    rdv.close()
    return 0


def single_gpu_same_job(ctx, args, tr, times_all, counts_all, steps, warmup):
    """Rank 0, after the sharded run: the same whole job on this one GPU (the 1-GPU denominator of
    the scaling claim, same config, same issue mode, same step).  Returns its line fragment."""
    b_in = ctx.batch(counts_all, with_time=args.mode != "frame")
    b_out = ctx.batch(counts_all)
    try:
        b_in.synth(seed=0, frame_id_base=1000)
        b_in.set_frame_times(times_all)
        if args.mode == "imu":
            b_in.set_frame_starts((times_all * 1e9).astype(np.int64))
        rdv1 = mc.dist.Rendezvous(0, 1)
        spun = 0.0
        if not args.no_tune:
            spun = spin_up(ctx, args.mode, b_in, b_out, args.spinup_ms / 2, args.issue)
            tune(ctx, args.mode, b_in, b_out)
        spin_up(ctx, args.mode, b_in, b_out, args.spinup_ms / 2 if spun else args.spinup_ms, args.issue)
        wall, tm, _ = run_mode(ctx, rdv1, args.mode, b_in, b_out, steps, warmup, issue=args.issue)
        n = int(counts_all.sum())
        kern = tm["main_ms"] / max(tm["main_launches"], 1) / 1e3
        return {"value": n * steps / wall / 1e6, "unit": "Mpoints/s", "ms_per_step": wall / steps * 1e3,
                "kernel_avg_us": kern * 1e6, "frac": BYTES_PER_POINT[args.mode] * n / kern / 1e9 / HBM_PEAK_GBS,
                "points": n, "steps": steps,
                "what": "the whole job (all frames of the config) on rank 0's GPU alone, after the sharded run"}
    finally:
        b_in.close()
        b_out.close()


def assemble_line(args, cid, label, scen, lo, hi, world, n_devices, n_rank, n_total, counts_all, results, spinup_ms,
                  every, tuned, stager, scan, codecs, parity, gather, hung, single) -> dict:
    """Rank 0's JSON line.  ``value`` is the timed steps' points over the max-over-ranks wall time
    (the kernels only: the merged-cloud gather runs after and outside the timed region and is
    reported on its own under ``gather``); at N > 1 the same-job single-GPU run and the speedup over
    it sit beside it (kernel scaling and gather reported separately)."""
    F_all = len(counts_all)
    r = results[args.mode]
    per_gpu_frames = hi - lo
    traffic, traffic_src = load_traffic(args.mode, per_gpu_frames, int(counts_all[0]) if F_all else 0)
    shared = n_devices < world
    scaling = "weak" if cid is None else "strong"
    gather_ok = None if gather is None else bool("error" not in gather and gather.get("parity", {}).get("ok"))
    ok = (gather_ok is not False) and (parity is None or parity["ok"]) and not hung
    line = {
        "metric": "Mpoints/s deskewed (100k-pt Mid-70 frames) + % HBM roofline",
        "value": r["value"],
        "unit": "Mpoints/s",
        "n_gpus": n_devices,
        "steps": r["steps"],
        "warmup": args.warmup,
        "spinup": {"ms": round(spinup_ms, 1), "what": "untimed, before the warmup steps: the same step "
                   "repeated until the device reaches its sustained memory throughput (tens of ms from "
                   "idle; 5 warmup steps are 1.7 ms) — profiles/round2/s51"},
        "ms_per_step": r["wall_s"] / r["steps"] * 1e3,
        "higher_is_better": True,
        "scaling": scaling if not shared else f"{scaling} (NOT a scaling result: {world} ranks share "
                                              f"{n_devices} device(s))",
        "vs_baseline": None,
        "dtype": "f64 arithmetic on f32 point columns (one f32 rounding per output coordinate)",
        "data": f"synthetic Mid-70 frames (counter-hash generator, on device); reference {scen} pose table, "
                "seed 42, GPS/IMU noise on",
        "config": {"workload": f"{label}; {world} rank(s), frames {lo}..{hi - 1} on rank 0",
                   "baseline_config": cid, "scenario": scen, "mode": args.mode,
                   "global_frames": F_all, "points_per_frame": int(counts_all[0]) if F_all else 0,
                   "total_points": n_total, "rank0_frames": per_gpu_frames,
                   "parallelism": f"frame-shard x{world} (dist.plan_shards)", "ranks": world,
                   "devices": n_devices},
        "roofline": {"bound": "hbm", "achieved": r["achieved_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": r["achieved_GBs"] / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": KERNEL_OF[args.issue][args.mode], "kernel_avg_us": r["main_avg_us"],
                     "kernel_each_us": r.get("main_span_us") or r.get("main_each_us"),
                     "events_avg_us": r.get("events_avg_us"), "events_each_us": r.get("main_each_us"),
                     "bytes_per_point": BYTES_PER_POINT[args.mode], "points_per_launch": n_rank,
                     "kernel_time": ("HIP events around every launch of a second, untimed pass"
                                     if args.events_after else
                                     (f"the kernels' own workgroup spans (first workgroup start to last "
                                      f"workgroup end, device wall clock) of {r['timed_launches']} of the "
                                      f"{r['steps']} timed steps (every {every}th); HIP events on the same "
                                      f"launches in events_* (they also hold the dispatch gap ahead of a launch)"
                                      if r.get("main_span_us") else
                                      f"HIP events (hipExtLaunchKernel start/stop) on the kernels of "
                                      f"{r['timed_launches']} of the {r['steps']} timed steps (every {every}th), "
                                      f"on the kernel's stream"))},
        "order_tune": tuned or None,
        "step_over_kernel": (r["wall_s"] / r["steps"] * 1e6) / r["main_avg_us"] if r["main_avg_us"] else None,
        "prep_avg_us": r["prep_avg_us"],
        "step_issue": {"calls": "per-call launches; prep as an any-order packet on the kernel's queue",
                       "pipeline": f"Context.deskew_steps: {r['steps'] + 1} launches, step 0's "
                                   "k_prep, then each step's deskew kernel with the next step's prep in its "
                                   "first workgroups (every step runs its own prep, one launch ahead)"}[args.issue],
        "modes": {m: {"Mpoints_s": v["value"], "kernel_GBs": v["achieved_GBs"],
                      "frac": v["achieved_GBs"] / HBM_PEAK_GBS, "kernel_avg_us": v["main_avg_us"],
                      "ms_per_step": v["wall_s"] / v["steps"] * 1e3}
                  for m, v in results.items()},
        "stager": stager,
        "scan_environment": scan,
        "codecs": codecs,
        "parity": parity,
        "gather": gather,
        "gather_ok": gather_ok,
        "single_gpu_same_job": single,
        "speedup_vs_1gpu": (r["value"] / single["value"]) if single and "value" in single else None,
        "ok": ok,
    }
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--spinup-ms", type=float, default=250.0,
                    help="untimed: run each mode's step for this long before its warmup steps (0: off)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", default="pose_slerp", choices=list(BYTES_PER_POINT))
    ap.add_argument("--config", default="auto", choices=["auto", "1", "2", "3", "4", "5"],
                    help="BASELINE config (auto: 2 at one GPU, 4 at N > 1)")
    ap.add_argument("--frames", type=int, default=None, help="custom job: frames per GPU (weak scaling)")
    ap.add_argument("--points", type=int, default=100_000, help="custom job: points per frame")
    ap.add_argument("--scenario", default="urban_complex", choices=list(SCENARIOS), help="custom job: pose table")
    ap.add_argument("--cpu-budget", type=float, default=6.0, help="seconds of CPU work per baseline leg")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="processes for the all-cores CPU legs (0: every core this process may use)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra-modes", action="store_true")
    ap.add_argument("--no-host-path", action="store_true", help="skip the host-array drop-in and save legs")
    ap.add_argument("--no-gather", action="store_true", help="skip the RCCL merged-cloud gather (N>1)")
    ap.add_argument("--no-check", action="store_true", help="skip the post-run oracle spot check (N=1)")
    ap.add_argument("--events-after", action="store_true",
                    help="per-launch HIP events in a second, untimed pass instead of the timed steps")
    ap.add_argument("--gather-timeout", type=float, default=300.0)
    ap.add_argument("--issue", choices=["pipeline", "calls"], default="pipeline",
                    help="how the timed steps are issued: pipeline = one Context.deskew_steps, each step's launch "
                         "also running the next step's prep; calls = one Context.deskew per step (prep + kernel)")
    ap.add_argument("--control-plane-only", action="store_true",
                    help="no GPU: the ranks rendezvous, allgather, max and barrier only (CPU test of the launch)")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="self-launch (--gpus N > 1 without torchrun): kill every rank after this many seconds")
    ap.add_argument("--no-single-gpu", action="store_true", help="N > 1: skip rank 0's same-job 1-GPU run")
    ap.add_argument("--no-tune", action="store_true", help="keep each mode's default sub-tile order (no mc_tune_order)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout))
    if args.control_plane_only:
        sys.exit(control_plane_only(args))

    rank, local_rank, world = mc.dist.env_rank()
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    rdv = mc.dist.Rendezvous(rank, world)
    cid, label, scen, cfg, tr, times_all, counts_all, lo, hi = workload(args, rank, world)
    times = times_all[lo:hi]
    counts = counts_all[lo:hi]
    cores = cpu_cores()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # before the GPU is initialised: the all-cores legs spawn worker processes
        procs = args.cpu_procs or cores["usable"]
        cpu = cpu_baselines(args.mode, tr, times, counts, lo, args.cpu_budget, procs)
        cpu["cores_visible"] = cores
    ctx = mc.Context()   # $MCDESKEW_DEVICE, else $LOCAL_RANK
    devices = rdv.allgather(ctx.pci_bus_id())
    n_devices = len(set(devices))

    b_in = ctx.batch(counts, with_time=True)
    b_out = ctx.batch(counts)
    b_in.synth(seed=0, frame_id_base=1000 + lo)
    # frame mode deskews the reference's (N,4) points (LMC:772-776): no t_ns column, 4 per block
    b_xyz = ctx.batch(counts)
    b_xyz.synth(seed=0, frame_id_base=1000 + lo)
    b_xyz.set_frame_times(times)
    b_in.set_frame_times(times)
    b_in.set_frame_starts((times * 1e9).astype(np.int64))
    ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
    ts_imu, gyro = mc.trajectory.imu_from_trajectory(tr, 200.0)
    ctx.set_imu(ts_imu, gyro)
    n_rank = int(counts.sum())
    n_total = int(counts_all.sum())
    src_of = {m: (b_xyz if m == "frame" else b_in) for m in BYTES_PER_POINT}

    modes = [args.mode] + ([] if args.no_extra_modes else [m for m in BYTES_PER_POINT if m != args.mode])
    results = {}
    tuned = {}
    every = 10
    for mode in modes:
        steps = args.steps if mode == args.mode else max(10, args.steps // 4)
        spun = 0.0
        if not args.no_tune and n_rank:
            # the orders are compared at sustained clocks: half the spin-up before the tuning (from
            # idle the first tens of ms run slow and decided the order by the ramp, profiles/round3/s48)
            spun += spin_up(ctx, mode, src_of[mode], b_out, args.spinup_ms / 2, args.issue)
            tuned[mode] = tune(ctx, mode, src_of[mode], b_out)
        spun += spin_up(ctx, mode, src_of[mode], b_out, args.spinup_ms / 2 if spun else args.spinup_ms, args.issue)
        if mode == args.mode:
            spinup_ms = spun
        wall, tm, ev = run_mode(ctx, rdv, mode, src_of[mode], b_out, steps, args.warmup,
                                live=not args.events_after, issue=args.issue)
        if mode == args.mode:
            every = ev
        wall_max = rdv.max(wall)
        events_avg_s = tm["main_ms"] / max(tm["main_launches"], 1) / 1e3
        spans = tm.get("main_span_us")
        main_avg_s = sum(spans) / len(spans) / 1e6 if spans else events_avg_s
        prep_avg_s = tm["prep_ms"] / tm["prep_launches"] / 1e3 if tm["prep_launches"] else None
        achieved = BYTES_PER_POINT[mode] * n_rank / main_avg_s / 1e9 if main_avg_s > 0 else 0.0
        results[mode] = {"wall_s": wall_max, "steps": steps, "main_avg_us": main_avg_s * 1e6,
                         "timed_launches": int(tm["main_launches"]), "main_each_us": tm["main_each_us"],
                         "main_span_us": spans, "events_avg_us": events_avg_s * 1e6,
                         "prep_avg_us": prep_avg_s * 1e6 if prep_avg_s is not None else None,
                         "achieved_GBs": achieved,
                         "value": n_total * steps / wall_max / 1e6}

    stager = measure_stager(ctx, b_xyz, b_out, n_rank, min(args.steps, 50)) if n_rank else None
    scan = codecs = None
    if not args.no_extra_modes and n_rank:
        scan = measure_scan(ctx, cfg, tr, 10, 0.0 if (args.no_cpu or world > 1) else 3.0)
        ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
        codecs = measure_codecs(ctx, src_of[args.mode], args.mode, b_out, n_rank, 5,
                                0.0 if (args.no_cpu or world > 1) else 1.0)
        codecs["pcd_ascii_fused"] = measure_deskew_pcd(ctx, src_of[args.mode], b_out, args.mode, n_rank, 5)
    imu = (ts_imu, gyro)
    F_all = len(counts_all)
    gather = parity = None
    hung = False
    if world > 1 and not args.no_gather:
        bounds = mc.dist.plan_shards(counts_all, world)
        sample = sorted({int(g) for r in range(world) if bounds[r + 1] > bounds[r]
                         for g in (bounds[r], (bounds[r] + bounds[r + 1]) // 2, bounds[r + 1] - 1)})

        def check(merged):
            return check_frames(merged, args.mode, tr, times_all, imu, counts_all, sample, sample)
        gather, hung = timed_gather(ctx, rdv, src_of[args.mode], b_out, args.mode, n_rank, world,
                                    args.gather_timeout, check)
    elif world == 1 and not args.no_check and F_all:
        ctx.deskew(src_of[args.mode], b_out, mode=args.mode)
        ctx.sync()
        loc = sorted({0, F_all // 2, F_all - 1})
        parity = check_frames(b_out, args.mode, tr, times_all, imu, counts_all, loc, loc)

    # the legs on the reference's own host-array calling convention load their own (urban_complex)
    # trajectories into the context: after the parity check, which deskews with the workload's
    host = save = None
    if world == 1 and not args.no_extra_modes and not args.no_host_path and n_rank:
        host = measure_host_path(ctx, cfg, len(counts), int(counts[0]) if len(counts) else 0, 3)
        save = measure_save(ctx)

    single = None
    if world > 1 and rank == 0 and not args.no_single_gpu and n_total:
        try:
            single = single_gpu_same_job(ctx, args, tr, times_all, counts_all, results[args.mode]["steps"],
                                         args.warmup)
        except Exception as e:  # reported in the line; the sharded result stands
            single = {"error": f"{type(e).__name__}: {e}"}

    ok = True
    if rank == 0:
        line = assemble_line(args, cid, label, scen, lo, hi, world, n_devices, n_rank, n_total, counts_all,
                             results, spinup_ms, every, tuned, stager, scan, codecs, parity, gather, hung, single)
        ok = line["ok"]
        if host is not None:
            line["host_path"] = host
            line["simulate_save"] = save
        if cpu is not None:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    if hung:
        # a collective is stuck inside RCCL: finalisers would block on its stream; the line is out
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)
    rdv.close()
    if not ok:
        sys.exit(4)


if __name__ == "__main__":
    main()
