set -u
OUT=gpurun_out/r3s74; mkdir -p $OUT
V=build/variants
for rep in 1 2 3; do
for l in fu2 fu1; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode frame --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('$l', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_avg_us'],1), d['order_tune']['frame']['chosen'], d['parity']['naive_rel_err']['coords_above_1e-5'])" | tee -a $OUT/bench.log
done; done
