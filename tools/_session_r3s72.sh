set -u
OUT=gpurun_out/r3s72; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$i.json'))
c=d['codecs']
print(round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_avg_us'],1), round(d['step_over_kernel'],4), {m: (round(v['frac'],4), round(v['kernel_avg_us'],1)) for m,v in d['modes'].items()}, 'lvx', round(c['lvx']['frac'],3), 'pcd', round(c['pcd_ascii']['frac'],3), 'fused', round(c['pcd_ascii_fused']['frac'],3), 'naive>1e-5', d['parity']['naive_rel_err']['coords_above_1e-5'])" | tee -a $OUT/bench_summary.log
done
