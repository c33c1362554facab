set -u
OUT=gpurun_out/r3s61; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab_pcd_fused.py --libs $V/lib_p1.so,$V/lib_p0.so > $OUT/ab_pcd_fused_order.log 2>&1 || exit $?
tail -8 $OUT/ab_pcd_fused_order.log
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --rounds 9 --libs $V/lib_p0.so,$V/lib_p1.so > $OUT/ab_codec_pcd_order.log 2>&1 || exit $?
grep median $OUT/ab_codec_pcd_order.log | head -2
