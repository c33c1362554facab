#!/bin/bash
# Instruction mix of the PCD passes (and the other codec / stager kernels) on the bench workload:
# one rocprofv3 --pmc pass of SQ counters over tools/aux_kernels.py (GPU box only).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pcd_pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PMC=${PMC_SET:-"SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU"}
timeout -s KILL 120 rocprofv3 --pmc $PMC \
  --output-format csv -d "$OUT/sq" -o run -- python3 "$ROOT/tools/aux_kernels.py" --reps 2 > "$OUT/sq.log" 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$ROOT/tools/aux_kernels.py" --reps 2 > "$OUT/trace.log" 2>&1 || exit 1
find "$OUT/trace" -name "*kernel_stats*" -exec cat {} \; | grep -E "pcd|lvx|soa|scan" | cut -d, -f1-4
python3 - "$OUT/sq" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    if any(s in k for s in ("pcd", "lvx", "soa", "scan")):
        print(k, {c: sum(x) / len(x) for c, x in v.items()})
PY
