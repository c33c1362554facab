set -u
OUT=gpurun_out/r3s43; mkdir -p $OUT
V=build/variants
for l in old ref old ref old ref; do
  for m in pose_slerp imu; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode $m --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench_${l}_$m.json 2> $OUT/bench_$l.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_${l}_$m.json'))
print('$l $m', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_avg_us'],1), round(d['step_over_kernel'],4))" | tee -a $OUT/bench.log
  done
done
