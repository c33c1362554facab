set -u
OUT=gpurun_out/r3s33; mkdir -p $OUT
V=build/variants
for l in f4 f2 f1 f4 f2 f1; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode frame --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench_$l.json 2> $OUT/bench_$l.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$l.json'))
print('$l', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'], json.dumps(d.get('order_tune')))" | tee -a $OUT/bench_frame.log
done
