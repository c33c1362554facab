set -u
OUT=gpurun_out/r3s67; mkdir -p $OUT
V=build/variants
timeout -k 10 700 python -u tools/ab_pcd_fused.py --modes pose_slerp,frame --libs $V/lib_t4.so,$V/lib_t8.so > $OUT/ab_pcd_tiles.log 2>&1 || exit $?
grep "fused frac" $OUT/ab_pcd_tiles.log
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --rounds 7 --libs $V/lib_t8.so,$V/lib_t4.so > $OUT/ab_codecs_tiles.log 2>&1 || exit $?
grep median $OUT/ab_codecs_tiles.log | head -3
