set -u
OUT=gpurun_out/r3s60; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
c=d['codecs']
print(round(d['value']), round(d['roofline']['frac'],4), {m: (round(v['frac'],4), round(v['kernel_avg_us'],1)) for m,v in d['modes'].items()}, 'lvx', round(c['lvx']['frac'],3), 'pcd', round(c['pcd_ascii']['frac'],3), 'fused', round(c['pcd_ascii_fused']['frac'],3))" | tee $OUT/bench_summary.log
