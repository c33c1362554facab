#!/bin/bash
# Where the hot kernels' waves spend their cycles: one rocprofv3 --pmc pass of SQ counters over the
# bench's three modes (GPU box only; separate pass from any kernel trace).
#   SQ_WAVE_CYCLES   wave-cycles resident        SQ_WAIT_ANY       wave-cycles waiting on anything
#   SQ_WAIT_INST_ANY waiting to issue            SQ_ACTIVE_INST_*  instructions issued, per type
# Usage (repo root):  bash tools/sq_modes.sh <tag>   -> gpurun_out/<tag>/sq_modes.log
set -u
TAG=${1:-sq}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PMC=${PMC_SET:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_ACTIVE_INST_LDS"}
timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d "$OUT/sq" -o run \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --spinup-ms 0 ${BENCH_ARGS:-} > "$OUT/sq_bench.log" 2>&1 || exit 1
python3 - "$OUT/sq" <<'PY' | tee "$OUT/sq_modes.log"
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    if "deskew" not in k:
        continue
    m = {c: sum(x) / len(x) for c, x in v.items()}
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    print(k, {c: f"{x:.4g}" for c, x in sorted(m.items())},
          f"wait/wave_cycles {m.get('SQ_WAIT_ANY', 0) / wc:.3f}",
          f"valu/wave_cycles {4 * m.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}")
PY
