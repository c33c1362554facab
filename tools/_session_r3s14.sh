set -u
OUT=gpurun_out/r3s14; mkdir -p $OUT
STEPS="tests" bash tools/gpu_session.sh r3s14 || exit $?
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$i.json'))
print(d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], json.dumps(d['order_tune']), {m: round(v['frac'],4) for m,v in d['modes'].items()})"
done
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-tune --no-cpu > $OUT/bench_notune.json 2> $OUT/bench_notune.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_notune.json'))
print('notune', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], {m: round(v['frac'],4) for m,v in d['modes'].items()})"
