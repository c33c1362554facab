set -u
OUT=gpurun_out/r3s24; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --libs $V/lib_cnl0.so,$V/lib_cnl1.so > $OUT/ab_codec_ntload.log 2>&1 || exit $?
tail -3 $OUT/ab_codec_ntload.log
timeout -k 10 600 python -u tools/ab_stager.py --replicas 2 --libs $V/lib_st1.so,$V/lib_st4.so,$V/lib_st0.so > $OUT/ab_stager_st.log 2>&1 || exit $?
python3 -c "
import json,re
t=open('$OUT/ab_stager_st.log').read(); d=json.loads(t[t.index('{'):])
print({k:(round(v['soa_to_aos']['median_us'],1), round(v['aos_to_soa']['median_us'],1)) for k,v in d.items()})"
