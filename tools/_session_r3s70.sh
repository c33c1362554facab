set -u
OUT=gpurun_out/r3s70; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --rounds 7 --libs $V/lib_mw0.so,$V/lib_mw1.so > $OUT/ab_pcd_measure.log 2>&1 || exit $?
grep median $OUT/ab_pcd_measure.log | head -2
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --rounds 7 --libs $V/lib_mw1.so,$V/lib_mw0.so > $OUT/ab_pcd_measure_b.log 2>&1 || exit $?
grep median $OUT/ab_pcd_measure_b.log | head -2
