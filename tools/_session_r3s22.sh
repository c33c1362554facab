set -u
OUT=gpurun_out/r3s22; mkdir -p $OUT
STEPS="tests smoke" bash tools/gpu_session.sh r3s22 || exit $?
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$i.json'))
c=d['codecs']
print(d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'], json.dumps(d['order_tune']), {m: round(v['frac'],4) for m,v in d['modes'].items()}, 'lvx', round(c['lvx']['frac'],3), 'pcd', round(c['pcd_ascii']['frac'],3), 'fused', round(c['pcd_ascii_fused']['frac'],3))"
done
MCDESKEW_DEVICE=0 timeout -k 10 900 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-gather --no-cpu --launch-timeout 800 > $OUT/bench_2ranks.json 2> $OUT/bench_2ranks.err
echo "2-rank rc=$?"
python3 -c "
import json; d=json.load(open('$OUT/bench_2ranks.json'))
print(d['value'], d['n_gpus'], d['scaling'], d['config']['workload'], json.dumps(d['single_gpu_same_job'])[:400], d['speedup_vs_1gpu'], d['ok'])" || true
STEPS="prof" bash tools/gpu_session.sh r3s22 || exit $?
