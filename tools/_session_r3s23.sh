set -u
OUT=gpurun_out/r3s23; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab.py --modes imu --replicas 3 --rounds 5 \
  --libs $V/lib_imu0.so,$V/lib_imu1.so,$V/lib_imuh.so > $OUT/ab_imu_r1.log 2>&1 || exit $?
grep replicas $OUT/ab_imu_r1.log
for l in imu0 imu1 imuh imu0 imu1 imuh; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode imu --no-extra-modes --no-cpu --steps 20 --warmup 5 > $OUT/bench_$l.json 2> $OUT/bench_$l.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$l.json'))
print('$l', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'], json.dumps(d['order_tune']))"
done
