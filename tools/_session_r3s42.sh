set -u
OUT=gpurun_out/r3s42; mkdir -p $OUT
V=build/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
tail -1 $OUT/pytest_gpu.log
MCDESKEW_LIB=$PWD/$V/lib_pair.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_pair.log 2>&1 || exit $?
tail -1 $OUT/pytest_gpu_pair.log
timeout -k 10 900 python -u tools/ab.py --modes pose_slerp,imu --replicas 2 --rounds 5 --check \
  --libs $V/lib_old.so,$V/lib_ref.so,$V/lib_pair.so > $OUT/ab_pair.log 2>&1 || exit $?
grep -E "replicas|differ" $OUT/ab_pair.log
for l in ref pair ref pair ref pair; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode pose_slerp --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench_$l.json 2> $OUT/bench_$l.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$l.json'))
print('$l', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'], d['parity']['naive_rel_err']['coords_above_1e-5'], json.dumps(d['order_tune']))" | tee -a $OUT/bench_slerp.log
done
