set -u
OUT=gpurun_out/s06; mkdir -p $OUT
STEPS="tests" bash tools/gpu_session.sh s06 || exit $?
V=build/variants
timeout -k 10 900 python -u tools/ab.py --modes pose_slerp,imu,frame --replicas 3 --rounds 5 \
  --libs $V/lib_r2f32.so,$V/lib_cur.so,$V/lib_s5.so,$V/lib_nopre.so > $OUT/ab.log 2>&1 || exit $?
cp gpurun_out/ab.json $OUT/ab.json
grep replicas $OUT/ab.log
STEPS="bench" bash tools/gpu_session.sh s06 || exit $?
