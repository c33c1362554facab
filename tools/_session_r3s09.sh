set -u
OUT=gpurun_out/r3s09; mkdir -p $OUT
V=build/variants
STEPS="tests" bash tools/gpu_session.sh r3s09 || exit $?
timeout -k 10 600 python -u tools/ab.py --modes pose_slerp --replicas 3 --rounds 5 \
  --libs $V/lib_cur.so,$V/lib_slerpd.so > $OUT/ab_slerp.log 2>&1 || exit $?
cp gpurun_out/ab.json $OUT/ab_slerp.json; grep replicas $OUT/ab_slerp.log
timeout -k 10 600 python -u tools/ab_stager.py --replicas 2 \
  --libs $V/lib_su1.so,$V/lib_su2.so,$V/lib_su4.so,$V/lib_su2pl.so > $OUT/ab_stager.log 2>&1 || exit $?
tail -12 $OUT/ab_stager.log
timeout -k 10 600 python -u tools/pingpong.py --modes pose_slerp,imu --rounds 4 --steps 12 \
  --arms same,fread,fwrite,flush,f256,fslerp,fidle \
  --libs $PWD/livox-motion-compensation-sim_amd/libmcdeskew.so,$PWD/$V/lib_slerpd.so \
  --out $OUT/pingpong.json > $OUT/pingpong.log 2>&1 || exit $?
cat $OUT/pingpong.log
STEPS="bench" bash tools/gpu_session.sh r3s09 || exit $?
