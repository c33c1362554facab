#!/bin/bash
# Step-issue A/B on one box: bench lines (K=20 and K=100) and rocprofv3 kernel-trace timelines
# (tools/step_timeline.py) for the MC_PREP_ISSUE variants built by
#   make -C livox-motion-compensation-sim_amd/csrc variants VARIANTS="issue0:-DMC_PREP_ISSUE=0 issue1:... issue2:..."
# plus the step graph (--graph).  Stops at the first failing step.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/issue_ab
mkdir -p "$OUT"
cd "$ROOT"
V=$ROOT/build/variants
for rep in 1 2; do
  for v in issue0 issue1 issue2; do
    for k in 20 100; do
      MCDESKEW_LIB=$V/lib_$v.so timeout -k 10 120 python bench.py --steps $k --no-cpu --no-extra-modes --no-check \
        > "$OUT/bench_${v}_k${k}_$rep.json" 2> "$OUT/bench_${v}_k${k}_$rep.err" || exit 1
      python -c "import json;d=json.load(open('$OUT/bench_${v}_k${k}_$rep.json'));print('$v k=$k rep=$rep', round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_avg_us'],1), round(d['step_over_kernel'],4))"
    done
  done
  timeout -k 10 120 python bench.py --steps 100 --no-cpu --no-extra-modes --no-check --graph > "$OUT/bench_graph_$rep.json" 2> "$OUT/bench_graph_$rep.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/bench_graph_$rep.json'));print('graph k=100 rep=$rep', round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_avg_us'],1), round(d['step_over_kernel'],4))"
done
cd /tmp && export TMPDIR=/tmp
for v in issue0 issue2; do
  MCDESKEW_LIB=$V/lib_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl_$v" -o run \
    -- python3 "$ROOT/bench.py" --steps 30 --no-cpu --no-extra-modes --no-check > "$OUT/tl_$v.json" 2> "$OUT/tl_$v.err" || exit 1
  python3 "$ROOT/tools/step_timeline.py" "$OUT/tl_$v/**/run_kernel_trace.csv" --label "$v" || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl_graph" -o run \
  -- python3 "$ROOT/bench.py" --steps 30 --no-cpu --no-extra-modes --no-check --graph > "$OUT/tl_graph.json" 2> "$OUT/tl_graph.err" || exit 1
python3 "$ROOT/tools/step_timeline.py" "$OUT/tl_graph/**/run_kernel_trace.csv" --label graph
