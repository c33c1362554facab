set -u
OUT=gpurun_out/r3s73; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --rounds 7 --libs $V/lib_cur.so,$V/lib_mt8.so,$V/lib_pf0.so > $OUT/ab_pcd_a.log 2>&1 || exit $?
grep median $OUT/ab_pcd_a.log | head -3
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --rounds 7 --libs $V/lib_pf0.so,$V/lib_mt8.so,$V/lib_cur.so > $OUT/ab_pcd_b.log 2>&1 || exit $?
grep median $OUT/ab_pcd_b.log | head -3
