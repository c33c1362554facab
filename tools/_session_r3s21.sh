set -u
OUT=gpurun_out/r3s21; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab.py --modes imu --replicas 3 --rounds 5 \
  --libs $V/lib_imu0.so,$V/lib_imu1.so > $OUT/ab_imu_r1.log 2>&1 || exit $?
grep replicas $OUT/ab_imu_r1.log
timeout -k 10 900 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-gather --no-cpu --launch-timeout 800 > $OUT/bench_2ranks.json 2> $OUT/bench_2ranks.err
echo "2-rank rc=$?"
python3 -c "
import json; d=json.load(open('$OUT/bench_2ranks.json'))
print(d['value'], d['n_gpus'], d['scaling'], d['config']['workload'], json.dumps(d['single_gpu_same_job'])[:300], d['speedup_vs_1gpu'])" || true
timeout -k 10 1200 python -u tools/bench_configs.py --out $OUT/configs.json > $OUT/configs.log 2>&1 || exit $?
cat $OUT/configs.log
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --libs $V/lib_cst0.so,$V/lib_cst1.so > $OUT/ab_codec_nt.log 2>&1 || exit $?
tail -3 $OUT/ab_codec_nt.log
