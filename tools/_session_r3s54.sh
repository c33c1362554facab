set -u
OUT=gpurun_out/r3s54; mkdir -p $OUT
V=build/variants
for rep in 1 2; do
for m in pose_slerp imu frame; do
for l in cur nl0; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode $m --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('$l $m', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_avg_us'],1), round(d['step_over_kernel'],4), d['order_tune']['$m']['chosen'], d['parity']['naive_rel_err']['coords_above_1e-5'])" | tee -a $OUT/bench.log
done; done; done
