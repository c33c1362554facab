set -u
OUT=gpurun_out/r3s26; mkdir -p $OUT
V=build/variants
timeout -k 10 900 python -u tools/ab.py --modes imu,pose_slerp --replicas 3 --rounds 5 \
  --libs $V/lib_base.so,$V/lib_null.so > $OUT/ab_nullmath.log 2>&1 || exit $?
grep replicas $OUT/ab_nullmath.log
