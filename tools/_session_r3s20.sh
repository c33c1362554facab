set -u
OUT=gpurun_out/r3s20; mkdir -p $OUT
STEPS="tests smoke" bash tools/gpu_session.sh r3s20 || exit $?
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$i.json'))
print(d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'], json.dumps(d['order_tune']), {m: round(v['frac'],4) for m,v in d['modes'].items()}, d['codecs']['pcd_ascii_fused']['frac'])"
done
STEPS="prof" bash tools/gpu_session.sh r3s20 || exit $?
timeout -k 10 300 python -u tools/latency.py > $OUT/latency.json 2> $OUT/latency.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/latency.json'))
print({k: (round(v['gap_us'],1), round(v['async_gap_us'],1), v['async_prep_launches']) for k,v in d['mc_deskew_per_call'].items()})"
