#!/bin/bash
# Occupancy cap sweep of the per-point kernels (dynamic LDS reserved per workgroup through
# $MCDESKEW_POINTS_LDS: 0 = 4 waves / SIMD, 49152 = 3, 61440 = 2) at two batch sizes, two processes
# each (placement varies per process).  GPU box only.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/occ_sweep
mkdir -p "$OUT"
cd "$ROOT"
for F in ${FRAMES:-600 3000}; do
  for rep in 1 2; do
    for L in 0 49152 61440; do
      for M in ${MODES:-pose_slerp imu}; do
        MCDESKEW_POINTS_LDS=$L timeout -k 10 240 python bench.py --frames $F --steps 20 --no-cpu --no-extra-modes \
          --no-check --mode $M > "$OUT/${M}_${F}_${L}_$rep.json" 2> "$OUT/${M}_${F}_${L}_$rep.err" || exit 1
        python -c "
import json; d=json.load(open('$OUT/${M}_${F}_${L}_$rep.json')); r=d['roofline']
print('$M', $F, $L, $rep, round(r['kernel_avg_us'],1), round(r['frac'],4), round(d['step_over_kernel'],4), flush=True)"
      done
    done
  done
done
