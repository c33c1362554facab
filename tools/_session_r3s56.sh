set -u
OUT=gpurun_out/r3s56; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
tail -1 $OUT/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 600 python bench.py --mode imu --no-extra-modes --no-cpu --no-tune --steps 50 --warmup 5 > $OUT/bench_imu_notune.json 2> $OUT/bench.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_imu_notune.json'))
print('imu no-tune', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_avg_us'],1), d['parity']['naive_rel_err']['coords_above_1e-5'])" | tee -a $OUT/bench.log
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log
