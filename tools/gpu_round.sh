#!/bin/bash
# One GPU-box session: gpu tests -> smoke -> bench -> rocprofv3 kernel trace.
# Stops at the first fault / abort / timeout (exit codes other than 0 and pytest's 1).
# Usage (from the repo root, on the GPU box):  bash tools/gpu_round.sh [tag] [steps]
# PMC=0 stops after the rocprof trace.  CONFIGS=1 adds the other BASELINE configs (tools/bench_configs.py) at the end.
set -u
TAG=${1:-r01}
STEPS=${2:-100}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"

stop_if_fault() {  # $1 = rc, $2 = step
  local rc=$1
  echo "[$2] rc=$rc" | tee -a "$OUT/steps_$TAG.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "[$2] fault/abort/timeout -> stopping" | tee -a "$OUT/steps_$TAG.log"
    exit "$rc"
  fi
}

timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --durations=0 --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
stop_if_fault $? pytest
tail -5 "$OUT/pytest_gpu_$TAG.log"

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
stop_if_fault $? smoke
cat "$OUT/smoke_$TAG.log"

timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 5 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
stop_if_fault $? bench
cat "$OUT/bench_$TAG.json"

cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run \
  -- python3 "$ROOT/bench.py" --steps "$STEPS" --no-cpu > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err"
stop_if_fault $? rocprof
find "$OUT/prof_$TAG" -name "*kernel_stats*" -exec cp {} "$OUT/kernel_stats_$TAG.csv" \;
# the bench line's roofline kernel time recomputed from the same run's kernel trace (timed window only)
python3 "$ROOT/tools/roofline_from_trace.py" --trace "$OUT/prof_$TAG" --bench "$OUT/prof_bench_$TAG.json" \
  --out "$OUT/roofline_trace_$TAG.json" > /dev/null 2>> "$OUT/prof_$TAG.err"
echo "[roofline_from_trace] rc=$?" | tee -a "$OUT/steps_$TAG.log"

cd "$ROOT"
if [ "${PMC:-1}" = "0" ]; then exit 0; fi
timeout -k 10 1200 python tools/pmc_traffic.py --tag "$TAG" > "$OUT/pmc_$TAG.log" 2>&1
stop_if_fault $? pmc
tail -5 "$OUT/pmc_$TAG.log"

timeout -k 10 900 python tools/pmc_traffic.py --aux --tag "$TAG" > "$OUT/pmc_aux_$TAG.log" 2>&1
stop_if_fault $? pmc_aux
tail -8 "$OUT/pmc_aux_$TAG.log"

if [ "${CONFIGS:-0}" = "1" ]; then
  timeout -k 10 900 python tools/bench_configs.py --out "$OUT/configs_$TAG.json" > "$OUT/configs_$TAG.log" 2>&1
  stop_if_fault $? configs
  cat "$OUT/configs_$TAG.log"
fi
