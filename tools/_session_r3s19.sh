set -u
OUT=gpurun_out/r3s19; mkdir -p $OUT
V=build/variants
STEPS="tests" bash tools/gpu_session.sh r3s19 || exit $?
MCDESKEW_LIB=$PWD/$V/lib_fuse.so timeout -k 10 600 python -u -m pytest tests/test_gpu_steps.py tests/test_gpu_parity.py -m gpu -q -x --timeout 240 --timeout-method thread > $OUT/pytest_fuse.log 2>&1 || exit $?
tail -2 $OUT/pytest_fuse.log
timeout -k 10 900 python -u tools/ab.py --modes pose_slerp --replicas 2 --rounds 5 \
  --libs $V/lib_nofuse.so,$V/lib_fuse.so,$V/lib_xfuse.so > $OUT/ab_fuse.log 2>&1 || exit $?
cp gpurun_out/ab.json $OUT/ab_fuse.json
grep -v replicas $OUT/ab_fuse.log | tail -6; grep replicas $OUT/ab_fuse.log
