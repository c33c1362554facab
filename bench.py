"""Benchmark: Mpoints/s deskewed + % of HBM roofline on synthetic Mid-70 100k-point frames.

One step = one pass of the hot path over one batch: the per-step pose prep (pose selection /
segment tables) + the deskew kernel over every point of the rank's 600 frames x 100k points
(BASELINE config 2: urban_complex, figure_eight).  Inputs are generated on the device and are
resident in HBM before the timed region.  Weak scaling: each rank owns 600 frames of a
600*N-frame urban_complex run (frames shard by index, no collective on the data path); the
RCCL gather of the merged cloud to rank 0 is timed separately after the steps.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode pose_slerp|frame|imu]
    torchrun --nproc-per-node N ... bench.py --gpus N   (one process per GPU, RCCL over xGMI)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import mcamd as mc  # noqa: E402

URBAN = {"duration": 120.0, "trajectory_type": "figure_eight", "environment_complexity": "complex",
         "max_speed": 12.0, "lidar_fps": 10}   # LMC:1183-1189
BYTES_PER_POINT = {"pose_slerp": 36, "imu": 36, "frame": 32}   # SURVEY §8d algorithmic bytes
HBM_PEAK_GBS = 8000.0                                          # MI355X_MICROARCH.md chip table


SCENARIOS = {   # LMC:1182-1204 (BASELINE configs 2 / 4 / 5: urban; 3: parking; 1: highway)
    "urban_complex": URBAN,
    "parking_detailed": {"duration": 30.0, "trajectory_type": "circular", "environment_complexity": "medium",
                         "max_speed": 5.0, "lidar_fps": 20},
    "highway_simple": {"duration": 60.0, "trajectory_type": "linear", "environment_complexity": "simple",
                       "max_speed": 25.0, "lidar_fps": 15},
}


def config_label(scenario, frames, points):
    if scenario == "urban_complex" and points >= 1_000_000:
        return "BASELINE config 5 shape: 1M-pt dense frames"
    return {"urban_complex": "BASELINE config 2 per GPU; config 4's frame shape at N GPUs (config 4 itself is "
                             "6000 frames = 750 per GPU at 8)", "parking_detailed": "BASELINE config 3",
            "highway_simple": "BASELINE config 1 scenario"}[scenario]


def workload(rank, world, frames, points, scenario="urban_complex"):
    base = SCENARIOS[scenario]
    cfg = dict(base, duration=max(base["duration"], frames * world / base["lidar_fps"]))
    sim = mc.LiDARMotionSimulator(cfg)
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()
    lo = rank * frames
    return cfg, tr, times[lo:lo + frames], lo


def _cpu_frames(mode, tr, times, counts, frame_lo, budget_s, f_first=0, f_step=1):
    """The oracle on frames f_first, f_first+f_step, ... until budget_s of compute; 1 BLAS thread.
    Returns (points, seconds, frames)."""
    from threadpoolctl import threadpool_limits
    from oracle import restatement as R
    from oracle import synth
    done = 0
    t_total = 0.0
    nf = 0
    ts_imu = gyro = None
    if mode == "imu":
        ts_imu, gyro = mc.trajectory.imu_from_trajectory(tr, 200.0)
    with threadpool_limits(limits=1):
        for f in range(f_first, len(counts), f_step):
            if t_total >= budget_s:
                break
            x, y, z, i, t = synth.synth_frame(int(counts[f]), 0, 1000 + frame_lo + f)
            pts = np.column_stack([x, y, z, i]).astype(np.float64)
            t0 = time.perf_counter()
            if mode == "frame":
                k = int(R.select_pose_index(tr["time"], times[f]))
                R.transform_pointcloud(pts, {"translation": tr["position_gps"][k], "rotation": tr["orientation_imu"][k]})
            elif mode == "pose_slerp":
                out = R.deskew_pose_slerp(pts[:, :3], t, times[f], tr)
                np.column_stack([out, pts[:, 3]])
            else:
                st = int(times[f] * 1e9)
                out = R.compensate_arrays(pts[:, :3], st + t.astype(np.int64), st, ts_imu, gyro)
                np.column_stack([out, pts[:, 3]])
            t_total += time.perf_counter() - t0
            done += int(counts[f])
            nf += 1
    return done, t_total, nf


def _cpu_worker(job):
    return _cpu_frames(*job)


def cpu_baselines(mode, tr, times, counts, frame_lo, budget_s, procs):
    """The oracle (numpy restatement of the reference's op sequence) on the same synthetic frames,
    generation excluded: one core, then `procs` processes (one BLAS thread each) splitting the
    frames round-robin.  Runs before the GPU is touched (the pool is spawned)."""
    import multiprocessing as mp
    done, secs, nf = _cpu_frames(mode, tr, times, counts, frame_lo, budget_s)
    single = {"value": done / secs / 1e6, "unit": "Mpoints/s", "cores": 1, "kind": "port",
              "sample": f"{nf} of {len(counts)} frames x {int(counts[0])} pts (oracle numpy restatement, "
                        f"same synthetic frames, generation excluded, {secs:.1f} s)"}
    if procs <= 1:
        return single
    jobs = [(mode, tr, times, counts, frame_lo, budget_s, p, procs) for p in range(procs)]
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(_cpu_worker, jobs)
    pts = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    frames = sum(r[2] for r in res)
    multi = {"value": pts / wall / 1e6, "unit": "Mpoints/s", "cores": procs, "kind": "port",
             "sample": f"{frames} of {len(counts)} frames x {int(counts[0])} pts over {procs} processes "
                       f"(1 BLAS thread each, round-robin frames), rate = points / slowest worker's compute time",
             "single_core": single}
    return multi



def aux_traffic(*kernels):
    """PMC traffic / algorithmic bytes of the kernels around the path (tools/pmc_traffic.py --aux)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    got = {k: d[f"aux:{k}"]["traffic_over_algorithmic"] for k in kernels if f"aux:{k}" in d}
    return got or None


def load_traffic(mode, frames, points):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    e = d.get(f"{mode}:{frames}x{points}")
    return None if e is None else e.get("hbm_bytes_per_launch")


def run_mode(ctx, rdv, mode, b_in, b_out, steps, warmup, live=True, graph=False):
    """Timed region: wall clock around ``steps`` steps.  ``live``: HIP events (no system-scope
    fence) around the kernels of every ``every``-th timed step themselves — on the stream each
    kernel is launched on — give the roofline's per-launch kernel time; events around every launch
    would cost ~2 % of the step rate (measured), sampling one step in ten ~0.2 %.  Otherwise a
    second, untimed pass carries events around every launch.  ``graph``: the ``steps`` steps are
    one replay of a HIP graph of ``steps`` deskew steps (``Context.deskew_steps``: every step runs
    its prep and kernel; the graph is captured before the timed region), else ``steps`` calls."""
    every = 10 if steps >= 50 else 5
    ctx.timing(live)           # warmup steps fill the context's event pool for the sampled steps
    for _ in range(warmup):
        ctx.deskew(b_in, b_out, mode=mode)
    if graph:                  # capture + instantiate only (host work, untimed)
        ctx.deskew_steps(b_in, b_out, steps, mode=mode, sample_every=every if live else 0, prepare=True)
    ctx.sync()
    ctx.timing(False)
    ctx.read_timing()          # drop the warmup events (back to the pool)
    rdv.barrier()
    t0 = time.perf_counter()
    if graph:
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
        ctx.timing(True)
        for _ in range(min(steps, 50)):
            ctx.deskew(b_in, b_out, mode=mode)
        ctx.sync()
        ctx.timing(False)
    tm = ctx.read_timing()
    return t1 - t0, tm


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
    times = mc.trajectory.lidar_times(cfg)[:1200]
    F = len(times)
    scfg = dict(mc.default_config(), **URBAN)
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


def measure_codecs(ctx, b_out, n_rank, reps, cpu_budget):
    """SURVEY §8f row 3, reported beside the hot path: the byte-exact writers (LVX v1.1 LMC:24-272,
    ASCII PCD LMC:932-948) encoding the rank's whole deskewed batch straight from its float32
    columns in HBM (mc_*_encode_batch).  Kernel time only (HIP events); HBM bytes = 16 B/pt read +
    the encoded bytes written."""
    from ctypes import c_int64, c_uint64
    counts = np.ascontiguousarray(b_out.counts, np.int64)
    F = len(counts)
    rep = {}
    pos = mc.codecs.lvx_layout(counts)
    ids = np.arange(F, dtype=np.uint64)
    ts = (np.arange(F) * 100_000_000).astype(np.uint64)
    out = ctx.device_buffer(int(pos[-1]))
    ptr = mc._lib.ptr

    def lvx():
        mc._lib.check(ctx.lib.mc_lvx_encode_batch(ctx.handle, b_out.handle, ptr(ids, c_uint64), ptr(ts, c_uint64),
                                                  out.ptr, int(pos[-1])), "lvx_encode_batch")
    lvx()
    ctx.read_timing()
    ctx.timing(True)
    for _ in range(reps):
        lvx()
    ctx.timing(False)
    ms = ctx.read_timing()["codec_ms"] / reps
    out.close()
    alg = 16 * n_rank + int(pos[-1])
    rep["lvx"] = {"file_bytes": int(pos[-1]), "kernels_ms": ms, "Mpoints_s": n_rank / ms / 1e3,
                  "GBs": alg / ms / 1e6, "frac": alg / ms / 1e6 / HBM_PEAK_GBS,
                  "bytes_per_point": alg / n_rank, "traffic_over_algorithmic": aux_traffic("k_lvx_packages")}
    bpos = np.zeros(F + 1, np.int64)
    cap = n_rank * 48
    out = ctx.device_buffer(cap)

    def pcd():
        mc._lib.check(ctx.lib.mc_pcd_encode_batch(ctx.handle, b_out.handle, out.ptr, cap, ptr(bpos, c_int64)),
                      "pcd_encode_batch")
    pcd()
    ctx.read_timing()
    ctx.timing(True)
    for _ in range(reps):
        pcd()
    ctx.timing(False)
    ms = ctx.read_timing()["codec_ms"] / reps
    out.close()
    text = int(bpos[-1])
    alg = 16 * n_rank + text
    rep["pcd_ascii"] = {"text_bytes": text, "kernels_ms": ms, "Mpoints_s": n_rank / ms / 1e3,
                        "GBs": alg / ms / 1e6, "frac": alg / ms / 1e6 / HBM_PEAK_GBS,
                        "bytes_per_point": alg / n_rank, "note": "measure + write passes",
                        "traffic_over_algorithmic": aux_traffic("k_pcd_measure", "k_pcd_write")}
    if cpu_budget > 0:
        from oracle import codecs as C
        host = b_out.download_aos()[:int(counts[0])]
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


def timed_gather(ctx, rdv, b_in, b_out, mode, n_rank, world, timeout_s):
    """The merged-cloud gather to rank 0 (LMC:887-889 over RCCL), after and outside the timed
    steps, under a watchdog so that a stuck collective can never cost the throughput line.
    Returns (report, hung).  The root's wall time is the gather time (it receives every shard)."""
    import threading
    res = {}

    def work():
        try:
            comm = mc.dist.RcclComm(ctx, rdv)
            ctx.deskew(b_in, b_out, mode=mode)
            ctx.sync()
            rdv.barrier()
            t0 = time.perf_counter()
            merged = mc.dist.gather_merged(ctx, comm, rdv, b_out, root=0)
            dt = time.perf_counter() - t0
            moved = 16 * n_rank * (world - 1)
            res["report"] = {"seconds": dt, "bytes_into_root": moved, "GBs": moved / dt / 1e9,
                             "merged_points": int(n_rank * world), "timed_on": "root wall clock"}
            if merged is not None:
                merged.close()
            comm.close()
        except Exception as e:  # report, never fail the throughput line
            res["report"] = {"error": str(e)}

    th = threading.Thread(target=work, daemon=True)
    th.start()
    th.join(timeout_s)
    if th.is_alive():
        return {"error": f"gather did not finish within {timeout_s} s"}, True
    return res.get("report"), False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", default="pose_slerp", choices=list(BYTES_PER_POINT))
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU baseline work (per process)")
    ap.add_argument("--cpu-procs", type=int, default=16, help="processes for the all-cores CPU baseline "
                    "(the box's CPU share per GPU)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra-modes", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="skip the RCCL merged-cloud gather (N>1)")
    ap.add_argument("--events-after", action="store_true",
                    help="per-launch HIP events in a second, untimed pass instead of the timed steps")
    ap.add_argument("--gather-timeout", type=float, default=120.0)
    ap.add_argument("--graph", action="store_true",
                    help="issue the timed steps as one HIP-graph replay (Context.deskew_steps; kernel time from "
                         "wall-clock stamp nodes, not HIP events) instead of separate calls")
    ap.add_argument("--scenario", default="urban_complex", choices=list(SCENARIOS),
                    help="pose table of this LMC scenario (BASELINE config 3 = parking_detailed)")
    args = ap.parse_args()

    rank, local_rank, world = mc.dist.env_rank()
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    rdv = mc.dist.Rendezvous(rank, world)
    cfg, tr, times, lo = workload(rank, world, args.frames, args.points, args.scenario)
    counts = np.full(args.frames, args.points, dtype=np.int64)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # before the GPU is initialised: the all-cores leg spawns worker processes
        cpu = cpu_baselines(args.mode, tr, times, counts, lo, args.cpu_budget,
                            min(args.cpu_procs, len(os.sched_getaffinity(0))))
        cpu["cores_available"] = len(os.sched_getaffinity(0))
    ctx = mc.Context()   # $MCDESKEW_DEVICE, else $LOCAL_RANK

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

    modes = [args.mode] + ([] if args.no_extra_modes else [m for m in BYTES_PER_POINT if m != args.mode])
    results = {}
    for mode in modes:
        steps = args.steps if mode == args.mode else max(10, args.steps // 4)
        wall, tm = run_mode(ctx, rdv, mode, b_xyz if mode == "frame" else b_in, b_out, steps, args.warmup,
                            live=not args.events_after, graph=args.graph)
        wall_max = rdv.max(wall)
        main_avg_s = tm["main_ms"] / max(tm["main_launches"], 1) / 1e3
        prep_avg_s = tm["prep_ms"] / max(tm["prep_launches"], 1) / 1e3
        achieved = BYTES_PER_POINT[mode] * n_rank / main_avg_s / 1e9
        results[mode] = {"wall_s": wall_max, "steps": steps, "main_avg_us": main_avg_s * 1e6,
                         "timed_launches": int(tm["main_launches"]),
                         "prep_avg_us": prep_avg_s * 1e6, "achieved_GBs": achieved,
                         "value": n_rank * world * steps / wall_max / 1e6}

    stager = measure_stager(ctx, b_xyz, b_out, n_rank, min(args.steps, 50))
    scan = codecs = None
    if not args.no_extra_modes:
        scan = measure_scan(ctx, cfg, tr, 10, 0.0 if (args.no_cpu or world > 1) else 3.0)
        ctx.set_trajectory(tr["time"], tr["position_gps"], tr["orientation_imu"])
        ctx.deskew(b_in, b_out, mode=args.mode)
        codecs = measure_codecs(ctx, b_out, n_rank, 5, 0.0 if (args.no_cpu or world > 1) else 1.0)

    gather = None
    hung = False
    if world > 1 and not args.no_gather:
        gather, hung = timed_gather(ctx, rdv, b_xyz if args.mode == "frame" else b_in, b_out, args.mode, n_rank,
                                    world, args.gather_timeout)

    if rank == 0:
        r = results[args.mode]
        traffic = load_traffic(args.mode, args.frames, args.points)
        line = {
            "metric": "Mpoints/s deskewed (100k-pt Mid-70 frames) + % HBM roofline",
            "value": r["value"],
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": r["steps"],
            "warmup": args.warmup,
            "ms_per_step": r["wall_s"] / r["steps"] * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (f64 pose/angle setup)",
            "data": f"synthetic Mid-70 frames (counter-hash generator, on device); reference {args.scenario} "
                    "pose table, seed 42",
            "config": {"workload": f"{args.scenario} {cfg['trajectory_type']}, {args.frames} frames x {args.points} "
                                   f"pts per GPU ({config_label(args.scenario, args.frames, args.points)}; "
                                   f"weak scaling over {world} GPU)",
                       "scenario": args.scenario,
                       "mode": args.mode, "frames_per_gpu": args.frames, "points_per_frame": args.points,
                       "global_frames": args.frames * world, "parallelism": f"frame-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": r["achieved_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": r["achieved_GBs"] / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "kernel": {"pose_slerp": "k_deskew_points<1>", "imu": "k_deskew_points<2>",
                                    "frame": "k_deskew_frame"}[args.mode],
                         "kernel_avg_us": r["main_avg_us"], "bytes_per_point": BYTES_PER_POINT[args.mode],
                         "kernel_time": ("HIP events around every launch of a second, untimed pass"
                                         if args.events_after else
                                         f"wall-clock stamp nodes around the kernels of {r['timed_launches']} of the "
                                         f"{r['steps']} steps of the step graph (every 10th)"
                                         if args.graph else
                                         f"HIP events around the kernels of {r['timed_launches']} of the "
                                         f"{r['steps']} timed steps (every 10th), on the kernel's stream")},
            "prep_avg_us": r["prep_avg_us"],
            "step_issue": "per-call launches" if not args.graph else
                          f"one HIP-graph replay of {r['steps']} steps (prep + kernel per step)",
            "modes": {m: {"Mpoints_s": v["value"], "kernel_GBs": v["achieved_GBs"],
                          "frac": v["achieved_GBs"] / HBM_PEAK_GBS, "kernel_avg_us": v["main_avg_us"]}
                      for m, v in results.items()},
            "stager": stager,
            "scan_environment": scan,
            "codecs": codecs,
            "gather": gather,
        }
        if cpu is not None:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    if hung:
        # a collective is stuck inside RCCL: finalisers would block on its stream; the result
        # line is out, so leave without running them
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    rdv.close()


if __name__ == "__main__":
    main()
