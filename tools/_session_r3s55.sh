set -u
OUT=gpurun_out/r3s55; mkdir -p $OUT
MCDESKEW_DEVICE=0 timeout -k 10 900 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-gather --no-cpu --launch-timeout 800 > $OUT/bench_2ranks.json 2> $OUT/bench_2ranks.err
echo "2-rank rc=$?"
python3 -c "
import json; d=json.load(open('$OUT/bench_2ranks.json'))
print(d['value'], d['n_gpus'], d['scaling'], d['config']['workload'], json.dumps(d['single_gpu_same_job'])[:300], d['speedup_vs_1gpu'], d['ok'])" || true
MCDESKEW_DEVICE=0 timeout -k 10 900 python -u bench.py --gpus 2 --mode imu --steps 10 --warmup 2 --no-gather --no-cpu --launch-timeout 800 > $OUT/bench_2ranks_imu.json 2> $OUT/bench_2ranks_imu.err
echo "2-rank imu rc=$?"
python3 -c "
import json; d=json.load(open('$OUT/bench_2ranks_imu.json'))
print(d['value'], d['n_gpus'], d['config']['workload'], d['speedup_vs_1gpu'], d['ok'])" || true
