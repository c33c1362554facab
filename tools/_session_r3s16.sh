set -u
OUT=gpurun_out/r3s16; mkdir -p $OUT
STEPS="tests smoke" bash tools/gpu_session.sh r3s16 || exit $?
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$i.json'))
print(d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'], json.dumps(d['order_tune']), {m: round(v['frac'],4) for m,v in d['modes'].items()})"
done
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-tune --no-cpu > $OUT/bench_notune.json 2> $OUT/bench_notune.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_notune.json'))
print('notune', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'], {m: round(v['frac'],4) for m,v in d['modes'].items()})"
STEPS="prof" bash tools/gpu_session.sh r3s16 || exit $?
