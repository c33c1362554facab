set -u
OUT=gpurun_out/r3s41; mkdir -p $OUT
V=build/variants
for l in w4 w5 w4 w5 w4 w5; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode pose_slerp --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench_$l.json 2> $OUT/bench_$l.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$l.json'))
print('$l', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'], d['parity']['naive_rel_err']['coords_above_1e-5'], json.dumps(d['order_tune']))" | tee -a $OUT/bench_slerp.log
done
