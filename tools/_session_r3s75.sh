set -u
OUT=gpurun_out/r3s75; mkdir -p $OUT
V=build/variants
timeout -k 10 700 python -u tools/ab_stager.py --replicas 3 --libs $V/lib_b4.so,$V/lib_b8.so > $OUT/ab_stager_batch.log 2>&1 || exit $?
python3 -c "
import json
t=open('$OUT/ab_stager_batch.log').read(); d=json.loads(t[t.index('{'):])
for k,v in d.items(): print(k, {kk:(round(vv['median_us'],1), round(vv.get('frac_median',0),3)) for kk,vv in v.items() if isinstance(vv,dict)})"
