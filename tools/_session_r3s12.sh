set -u
OUT=gpurun_out/r3s12; mkdir -p $OUT
V=build/variants
PYTEST_ARGS="-k codecs" STEPS="tests" bash tools/gpu_session.sh r3s12 || exit $?
MCDESKEW_LIB=$PWD/$V/lib_pc1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_codecs.py -m gpu -k deskew_pcd -q -x --timeout 120 --timeout-method thread > $OUT/pytest_pc1.log 2>&1 || exit $?
tail -2 $OUT/pytest_pc1.log
timeout -k 10 600 python -u tools/ab_pcd_fused.py --libs $V/lib_pc0.so,$V/lib_pc1.so --modes pose_slerp,frame,imu > $OUT/ab_pcd_fused.log 2>&1 || exit $?
cat $OUT/ab_pcd_fused.log
timeout -k 10 300 python -u tools/latency.py > $OUT/latency.json 2> $OUT/latency.err || exit $?
cat $OUT/latency.json
timeout -k 10 600 python -u tools/ab.py --modes pose_slerp --replicas 3 --rounds 5 \
  --libs $V/lib_cur.so,$V/lib_slerpd.so,$V/lib_alt.so > $OUT/ab_slerp_alt.log 2>&1 || exit $?
grep replicas $OUT/ab_slerp_alt.log
