set -u
OUT=gpurun_out/r3s59; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --rounds 9 --libs $V/lib_cx0.so,$V/lib_cx1.so > $OUT/ab_codec_order_a.log 2>&1 || exit $?
grep median $OUT/ab_codec_order_a.log | head -2
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --rounds 9 --libs $V/lib_cx1.so,$V/lib_cx0.so > $OUT/ab_codec_order_b.log 2>&1 || exit $?
grep median $OUT/ab_codec_order_b.log | head -2
