set -u
OUT=gpurun_out/r3s49; mkdir -p $OUT
for m in frame frame frame frame imu imu pose_slerp pose_slerp; do
  timeout -k 10 600 python bench.py --mode $m --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench_$m.json 2> $OUT/bench_$m.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$m.json'))
print('$m', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_avg_us'],1), round(d['step_over_kernel'],4), json.dumps(d['order_tune']), d['parity']['naive_rel_err']['coords_above_1e-5'])" | tee -a $OUT/bench.log
done
