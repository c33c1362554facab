#!/bin/bash
# One GPU-box session, steps chosen by $STEPS (default: tests smoke ab bench), each under its own
# time limit; stops at the first fault / abort / timeout (any exit code other than 0 and pytest's 1).
#   tests   python -m pytest tests -m gpu ($PYTEST_ARGS, e.g. "-k slerp")
#   smoke   __graft_entry__.smoke()
#   ab      tools/ab.py $AB_ARGS (interleaved A/B of build/variants/lib_*.so)
#   bench   bench.py with the driver's flags ($BENCH_ARGS)
#   abc     tools/ab_codecs.py $ABC_ARGS (interleaved A/B of the codec kernels across libraries)
#   abf     tools/ab_pcd_fused.py $ABF_ARGS (interleaved A/B of the fused deskew -> PCD pipeline)
#   pcdpmc  tools/pcd_pmc.sh (SQ instruction counters of the codec / stager kernels)
#   pmc     tools/pmc_traffic.py (deskew kernels, then --aux), profiles/pmc_traffic.json copied out
#   latency tools/latency.py ($LAT_ARGS)
#   prof    rocprofv3 --kernel-trace --stats of the same bench command
#   smi     rocm-smi clocks / power / temperature appended to smi.log
#   probe   tools/issue_probe (issue cost of the codec kernels' vector / LDS instructions)
# Usage (repo root, on the GPU box):  STEPS="tests ab" bash tools/gpu_session.sh <tag>
set -u
TAG=${1:-s}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
STEPS=${STEPS:-"tests smoke ab bench"}

stop_if_fault() {  # $1 = rc, $2 = step
  echo "[$2] rc=$1 $(date +%T)" | tee -a "$OUT/steps.log"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then
    echo "[$2] fault/abort/timeout -> stopping" | tee -a "$OUT/steps.log"
    exit "$1"
  fi
}

for step in $STEPS; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -x --durations=15 --timeout 240 \
        --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
      stop_if_fault $? tests
      tail -25 "$OUT/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      stop_if_fault $? smoke
      cat "$OUT/smoke.log" ;;
    ab)
      timeout -k 10 900 python -u tools/ab.py ${AB_ARGS:-} > "$OUT/ab.log" 2>&1
      stop_if_fault $? ab
      cp gpurun_out/ab.json "$OUT/ab.json" 2>/dev/null
      cat "$OUT/ab.log" ;;
    bench)
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
      stop_if_fault $? bench
      cat "$OUT/bench.json"; tail -3 "$OUT/bench.err" ;;
    abc)
      timeout -k 10 600 python -u tools/ab_codecs.py ${ABC_ARGS:-} > "$OUT/ab_codecs.log" 2>&1
      stop_if_fault $? abc
      cat "$OUT/ab_codecs.log" ;;
    abf)
      timeout -k 10 600 python -u tools/ab_pcd_fused.py ${ABF_ARGS:-} > "$OUT/ab_fused.log" 2>&1
      stop_if_fault $? abf
      cat "$OUT/ab_fused.log" ;;
    pcdpmc)
      timeout -k 10 400 bash tools/pcd_pmc.sh > "$OUT/pcd_pmc.log" 2>&1
      stop_if_fault $? pcdpmc
      tail -8 "$OUT/pcd_pmc.log" ;;
    pmc)
      timeout -k 10 900 python tools/pmc_traffic.py --tag "$TAG" > "$OUT/pmc.log" 2>&1
      stop_if_fault $? pmc
      timeout -k 10 900 python tools/pmc_traffic.py --aux --tag "$TAG" > "$OUT/pmc_aux.log" 2>&1
      stop_if_fault $? pmc_aux
      cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
      tail -8 "$OUT/pmc_aux.log" ;;
    latency)
      timeout -k 10 300 python -u tools/latency.py ${LAT_ARGS:-} > "$OUT/latency.json" 2> "$OUT/latency.err"
      stop_if_fault $? latency
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: d[k] for k in d if k != 'mc_deskew_per_call'})" "$OUT/latency.json" ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu ${BENCH_ARGS:-} \
          > "$OUT/prof_bench.json" 2> "$OUT/prof.err" )
      stop_if_fault $? prof
      find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/kernel_stats.csv" \;
      head -12 "$OUT/kernel_stats.csv"
      # the bench line's roofline kernel time recomputed from the same run's kernel trace (timed window)
      python3 tools/roofline_from_trace.py --trace "$OUT/prof" --bench "$OUT/prof_bench.json" \
        --out "$OUT/roofline_trace.json" > /dev/null 2>> "$OUT/prof.err"
      echo "[roofline_from_trace] rc=$?" | tee -a "$OUT/steps.log" ;;
    smi)
      timeout -k 10 60 rocm-smi --showclocks --showpower --showtemp >> "$OUT/smi.log" 2>&1
      echo "---- $(date +%T)" >> "$OUT/smi.log" ;;
    probe)
      timeout -k 10 300 tools/issue_probe > "$OUT/issue_probe.json" 2> "$OUT/issue_probe.err"
      stop_if_fault $? probe
      cat "$OUT/issue_probe.json" ;;
    *) echo "unknown step $step" ;;
  esac
done
