"""Run bench.py on the other BASELINE.json configurations (one GPU) and collect their lines.

  config 1  highway_simple, 10 frames x 20k points
  config 3  parking_detailed, 600 x 100k (noise on; the SLERP-heavy pose table)
  config 4  the whole 6000 x 100k job on ONE GPU (600 M points; 8 GPUs shard it 750 per GPU)
  config 5  the whole 1200 x 1M-point job on ONE GPU (1.2 G points, 6.0 G input values > 2^32)
  config 5 shape  its per-GPU shape at 8 GPUs: 150 x 1M
  (configs 4 / 5 whole jobs also in frame mode: the reference's own transform_pointcloud, LMC:772-776)

Each run is a child process under its own time limit; the first failure ends the sweep.
Usage (GPU box):  python tools/bench_configs.py --out gpurun_out/configs.json
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = {
    "config1_highway_10x20k": ["--config", "1"],
    "config3_parking_600x100k": ["--config", "3"],
    "config4_whole_6000x100k_1gpu": ["--config", "4", "--no-extra-modes"],
    "config4_whole_6000x100k_1gpu_frame": ["--config", "4", "--no-extra-modes", "--mode", "frame"],
    "config5_whole_1200x1M_1gpu": ["--config", "5", "--no-extra-modes"],
    "config5_whole_1200x1M_1gpu_frame": ["--config", "5", "--no-extra-modes", "--mode", "frame"],
    "config5_shape_150x1M": ["--frames", "150", "--points", "1000000"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    res = {}
    for name, extra in CONFIGS.items():
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(args.steps), "--no-cpu"] + extra
        p = subprocess.run(["timeout", "-k", "10", "300"] + cmd, capture_output=True, text=True, cwd=ROOT)
        if p.returncode != 0:
            res[name] = {"error": p.returncode, "stderr": p.stderr[-2000:]}
            print(name, "failed", p.returncode, file=sys.stderr)
            break
        line = json.loads(p.stdout.strip().splitlines()[-1])
        res[name] = {"config": line["config"], "value_Mpoints_s": line["value"], "ms_per_step": line["ms_per_step"],
                     "modes": line["modes"], "roofline": line["roofline"], "parity": line.get("parity"),
                     "step_over_kernel": line.get("step_over_kernel"), "order_tune": line.get("order_tune")}
        print(name, {m: round(v["frac"], 4) for m, v in line["modes"].items()}, flush=True)
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0 if all("error" not in v for v in res.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
