set -u
OUT=gpurun_out/r3s58; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --libs $V/lib_cx1.so,$V/lib_cx0.so > $OUT/ab_codec_order.log 2>&1 || exit $?
grep median $OUT/ab_codec_order.log | head -4
