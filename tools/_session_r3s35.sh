set -u
OUT=gpurun_out/r3s35; mkdir -p $OUT
V=build/variants
timeout -k 10 900 python -u tools/ab.py --modes imu --replicas 3 --rounds 5 --check \
  --libs $V/lib_ib.so,$V/lib_iwf.so > $OUT/ab_imu_winfirst.log 2>&1 || exit $?
grep -E "replicas|differ" $OUT/ab_imu_winfirst.log
for l in ib iwf ib iwf ib iwf; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode imu --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench_$l.json 2> $OUT/bench_$l.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$l.json'))
print('$l', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'])" | tee -a $OUT/bench_imu.log
done
