#!/bin/bash
# Does the deskew kernels' HBM rate fall with batch size (BASELINE configs 4 / 5 whole jobs run at
# ~71 % of peak on one GPU vs ~83 % at 600 x 100k)?  Bench lines for 600..6000 x 100k frames, then
# TLB (UTCL1) and HBM traffic counters at 600 and 6000 frames (one --pmc pass each; GPU box only).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/size_sweep
mkdir -p "$OUT"
cd "$ROOT"
for F in 600 1200 2400 3600 6000; do
  timeout -k 10 180 python bench.py --frames $F --steps 20 --no-cpu --no-extra-modes --no-check --mode pose_slerp \
    > "$OUT/slerp_$F.json" 2> "$OUT/slerp_$F.err" || exit 1
  timeout -k 10 180 python bench.py --frames $F --steps 20 --no-cpu --no-extra-modes --no-check --mode frame \
    > "$OUT/frame_$F.json" 2> "$OUT/frame_$F.err" || exit 1
  python -c "
import json
for m in ('slerp','frame'):
    d=json.load(open('$OUT/'+m+'_$F.json')); r=d['roofline']
    print(m, $F, round(r['kernel_avg_us'],1), round(r['frac'],4), round(d['step_over_kernel'],4))"
done
cd /tmp && export TMPDIR=/tmp
for F in 600 6000; do
  for P in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_STALL_MULTI_MISS_sum" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE"; do
    tag=$(echo $P | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/pmc_${F}_$tag" -o run \
      -- python3 "$ROOT/bench.py" --frames $F --steps 4 --warmup 1 --no-cpu --no-extra-modes --no-check \
      > "$OUT/pmc_${F}_$tag.json" 2> "$OUT/pmc_${F}_$tag.err" || exit 1
    python3 - "$OUT/pmc_${F}_$tag" "$F" <<'PY'
import csv, glob, sys, statistics, collections
d = collections.defaultdict(list)
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        if "k_deskew_points<1" in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: statistics.median(v) for k, v in d.items()})
PY
  done
done
