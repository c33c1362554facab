set -u
OUT=gpurun_out/r3s48; mkdir -p $OUT
V=build/variants
for l in f4 f2 f4 f2 f4 f2 f4 f2; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode frame --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench_$l.json 2> $OUT/bench_$l.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$l.json'))
print('$l', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_avg_us'],1), round(d['step_over_kernel'],4), d['order_tune']['frame']['chosen'])" | tee -a $OUT/bench.log
done
