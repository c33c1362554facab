set -u
OUT=gpurun_out/r3s66; mkdir -p $OUT
V=build/variants
timeout -k 10 700 python -u tools/ab_pcd_fused.py --modes pose_slerp --libs $V/lib_t8.so,$V/lib_t4.so,$V/lib_t16.so > $OUT/ab_pcd_tiles.log 2>&1 || exit $?
grep "fused frac" $OUT/ab_pcd_tiles.log
