#!/bin/bash
# Per-TCC-channel DRAM request and credit-stall counters on fast vs slow replicas (tools/placement_pmc.py).
# One --pmc pass per raw counter (16 derived per-channel selects of it, tools/pmc/tcc_channels.yaml).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/placement
mkdir -p "$OUT"
MODE=${1:-frame}
cd /tmp && export TMPDIR=/tmp
for C in RD WR RDST WRST; do
  P=$(for i in $(seq 0 15); do printf "MC_%s_I%d " $C $i; done)
  timeout -s KILL 120 rocprofv3 -E "$ROOT/tools/pmc/tcc_channels.yaml" --pmc $P --output-format csv -d "$OUT/pmc_$C" -o run \
    -- python3 "$ROOT/tools/placement_pmc.py" --mode $MODE --times "$OUT/times_$C.json" > "$OUT/run_$C.log" 2>&1 || { tail -5 "$OUT/run_$C.log"; exit 1; }
  python3 "$ROOT/tools/placement_pmc.py" --mode $MODE --parse "$OUT/pmc_$C" --times "$OUT/times_$C.json" --out "$OUT/channels_$C.json" || exit 1
done
