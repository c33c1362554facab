set -u
OUT=gpurun_out/r3s36; mkdir -p $OUT
V=build/variants
MCDESKEW_LIB=$PWD/$V/lib_d1.so timeout -k 10 900 python -u -m pytest tests -m gpu -k "imu or IMU or compensate or steps" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_imu_d1.log 2>&1 || exit $?
tail -1 $OUT/pytest_imu_d1.log
timeout -k 10 900 python -u tools/ab.py --modes imu --replicas 3 --rounds 5 --check \
  --libs $V/lib_d0.so,$V/lib_d1.so > $OUT/ab_imu_swinperm.log 2>&1 || exit $?
grep -E "replicas|differ" $OUT/ab_imu_swinperm.log
for l in ib swp ib swp ib swp; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode imu --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench_$l.json 2> $OUT/bench_$l.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$l.json'))
print('$l', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'], d['parity']['naive_rel_err']['coords_above_1e-5'], d['order_tune']['imu']['chosen'])" | tee -a $OUT/bench_imu.log
done
