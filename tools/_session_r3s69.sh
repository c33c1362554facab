set -u
OUT=gpurun_out/r3s69; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --rounds 7 --libs $V/lib_u1.so,$V/lib_u2.so,$V/lib_u4.so > $OUT/ab_lvx_units.log 2>&1 || exit $?
grep median $OUT/ab_lvx_units.log | head -3
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --rounds 7 --libs $V/lib_u4.so,$V/lib_u2.so,$V/lib_u1.so > $OUT/ab_lvx_units_b.log 2>&1 || exit $?
grep median $OUT/ab_lvx_units_b.log | head -3
