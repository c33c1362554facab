"""Measure HBM traffic per launch of the hot kernels with rocprofv3 PMC counters (GPU box only).

Recipe (MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7): FETCH_SIZE and WRITE_SIZE in
separate --pmc passes (TCC slots cannot hold both), kernel trace only, no sys/runtime tracing;
FETCH_SIZE counts KiB and on gfx950 reports exactly half the bytes of a wide coalesced stream,
so it is doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.

    python tools/pmc_traffic.py [--tag r01] [--modes pose_slerp,frame,imu]

Writes profiles/pmc_traffic.json (read by bench.py as roofline.traffic) and keeps the raw
counter CSVs under gpurun_out/.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = {"pose_slerp": "k_deskew_points<1", "imu": "k_deskew_points<2", "frame": "k_deskew_frame"}
BYTES_PER_POINT = {"pose_slerp": 36, "imu": 36, "frame": 32}


def run_pass(mode, counter, outdir, frames, points):
    d = os.path.join(outdir, f"pmc_{mode}_{counter}")
    cmd = ["timeout", "-k", "10", "300", "rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d,
           "-o", "run", "--", sys.executable, os.path.join(ROOT, "bench.py"), "--mode", mode, "--steps", "10",
           "--warmup", "2", "--no-cpu", "--no-extra-modes", "--frames", str(frames), "--points", str(points)]
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-2000:] + r.stderr[-4000:])
        raise SystemExit(f"rocprofv3 pass {mode}/{counter} failed rc={r.returncode}")
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    vals = []
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if KERNEL[mode] in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {KERNEL[mode]} in {files}")
    return statistics.median(vals), len(vals)


AUX = ["k_soa_to_aos", "k_aos_to_soa", "k_lvx_packages", "k_pcd_measure", "k_pcd_write",
       "k_scan_count", "k_scan_emit"]


def run_aux(counter, outdir):
    """One counter pass over tools/aux_kernels.py; returns ({kernel: median KiB}, alg bytes)."""
    d = os.path.join(outdir, f"pmc_aux_{counter}")
    cmd = ["timeout", "-k", "10", "300", "rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d,
           "-o", "run", "--", sys.executable, os.path.join(ROOT, "tools", "aux_kernels.py")]
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-2000:] + r.stderr[-4000:])
        raise SystemExit(f"rocprofv3 aux pass {counter} failed rc={r.returncode}")
    alg = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])["algorithmic_bytes_per_launch"]
    vals = {k: [] for k in AUX}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                for k in AUX:
                    name = row.get("Kernel_Name", "")
                    if f"mc::{k}(" in name or f"mc::{k}<" in name:   # plain or templated kernel
                        vals[k].append(float(row["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items() if v}, alg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--aux", action="store_true", help="the kernels around the path (tools/aux_kernels.py)")
    ap.add_argument("--modes", default="pose_slerp,frame,imu")
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--points", type=int, default=100_000)
    ap.add_argument("--tag", default="r01")
    args = ap.parse_args()
    outdir = os.path.join(ROOT, "gpurun_out", f"pmc_{args.tag}")
    os.makedirs(outdir, exist_ok=True)
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    res = {}
    if os.path.exists(path):
        with open(path) as f:
            res = json.load(f)
    if args.aux:
        fetch, alg = run_aux("FETCH_SIZE", outdir)
        write, _ = run_aux("WRITE_SIZE", outdir)
        for k in AUX:
            if k not in fetch or k not in write:
                continue
            f_b, w_b = fetch[k] * 1024 * 2, write[k] * 1024
            res[f"aux:{k}"] = {"kernel": k, "fetch_bytes_per_launch": f_b, "write_bytes_per_launch": w_b,
                               "hbm_bytes_per_launch": f_b + w_b, "algorithmic_bytes_per_launch": alg[k],
                               "traffic_over_algorithmic": (f_b + w_b) / alg[k], "tag": args.tag,
                               "note": "tools/aux_kernels.py workload; FETCH_SIZE x2 (gfx950 correction)"}
            print(k, json.dumps(res[f"aux:{k}"]))
        args.modes = ""
    for mode in [m for m in args.modes.split(",") if m]:
        fetch_kib, n1 = run_pass(mode, "FETCH_SIZE", outdir, args.frames, args.points)
        write_kib, n2 = run_pass(mode, "WRITE_SIZE", outdir, args.frames, args.points)
        fetch = fetch_kib * 1024 * 2      # gfx950: FETCH_SIZE reports half of a wide coalesced read
        write = write_kib * 1024
        alg = BYTES_PER_POINT[mode] * args.frames * args.points
        res[f"{mode}:{args.frames}x{args.points}"] = {
            "kernel": KERNEL[mode], "dispatches": [n1, n2],
            "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
            "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
            "hbm_bytes_per_launch": fetch + write, "algorithmic_bytes_per_launch": alg,
            "traffic_over_algorithmic": (fetch + write) / alg, "tag": args.tag,
            "note": "rocprofv3 --pmc, separate FETCH_SIZE/WRITE_SIZE passes; FETCH_SIZE x2 (gfx950 correction)",
        }
        print(mode, json.dumps(res[f"{mode}:{args.frames}x{args.points}"]))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    for p in (path, os.path.join(ROOT, "gpurun_out", "pmc_traffic.json")):   # gpurun_out travels back
        with open(p, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
