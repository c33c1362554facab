"""Run bench.py on the other BASELINE.json configurations (one GPU) and collect their lines.

  config 1  highway_simple, 10 frames x 20k points
  config 3  parking_detailed, 600 x 100k (noise on; the SLERP-heavy pose table)
  config 5  the per-GPU shape of 1200 x 1M-point frames over 8 GPUs: 150 x 1M

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
    "config1_highway_10x20k": ["--scenario", "highway_simple", "--frames", "10", "--points", "20000"],
    "config3_parking_600x100k": ["--scenario", "parking_detailed", "--frames", "600", "--points", "100000"],
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
                     "modes": line["modes"]}
        print(name, {m: round(v["frac"], 4) for m, v in line["modes"].items()}, flush=True)
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0 if all("error" not in v for v in res.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
