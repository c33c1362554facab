set -u
OUT=gpurun_out/r3s44; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab_stager.py --replicas 3 --libs $V/lib_st1.so,$V/lib_st0.so,$V/lib_st3.so > $OUT/ab_stager_st.log 2>&1 || exit $?
python3 -c "
import json
t=open('$OUT/ab_stager_st.log').read(); d=json.loads(t[t.index('{'):])
for k,v in d.items(): print(k, {kk:(round(vv['median_us'],1), round(vv.get('frac_median',0),3)) for kk,vv in v.items() if isinstance(vv,dict)})"
