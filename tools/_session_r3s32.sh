set -u
OUT=gpurun_out/r3s32; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python bench.py --steps 50 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
python3 -c "
import json; d=json.load(open('$OUT/bench_default.json'))
print('default', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'], {m: round(v.get('frac',0),3) for m,v in d.get('modes',{}).items()} if isinstance(d.get('modes'),dict) else '')"
for l in p2 p4 p2 p4; do
  MCDESKEW_LIB=$PWD/$V/lib_$l.so timeout -k 10 600 python bench.py --mode pose_slerp --no-extra-modes --no-cpu --steps 50 --warmup 5 > $OUT/bench_$l.json 2> $OUT/bench_$l.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$l.json'))
print('$l', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['step_over_kernel'])" | tee -a $OUT/bench_slerp.log
done
