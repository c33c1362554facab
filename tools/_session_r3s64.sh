set -u
OUT=gpurun_out/r3s64; mkdir -p $OUT
V=build/variants
for rep in 1 2 3; do
for l in cur nofuse; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode pose_slerp --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('$l', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_avg_us'],1), round(d['ms_per_step']*1e3,1), round(d['step_over_kernel'],4), d['order_tune']['pose_slerp']['chosen'])" | tee -a $OUT/bench.log
done; done
