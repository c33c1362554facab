set -u
OUT=gpurun_out/r3s50; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --libs $V/lib_cnt1.so,$V/lib_csc1.so > $OUT/ab_codec_sc1.log 2>&1 || exit $?
tail -4 $OUT/ab_codec_sc1.log
timeout -k 10 600 python -u tools/ab_pcd_fused.py --libs $V/lib_cnt1.so,$V/lib_csc1.so > $OUT/ab_pcd_fused_sc1.log 2>&1 || exit $?
tail -6 $OUT/ab_pcd_fused_sc1.log
