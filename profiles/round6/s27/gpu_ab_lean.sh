# PCD text-length counting A/B (round 6, s27): the codec / PCD-length GPU tests on the lean build,
# then tools/ab_pcd_fused.py across the packed (MC_PCD_LEAN=0) and lean (=1) variant libraries.
set -u
OUT=gpurun_out/r6s27
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_codecs.py tests/test_gpu_scan.py tests/test_gpu_run.py -m gpu -x -q \
  --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 600 python -u tools/ab_pcd_fused.py --libs build/variants/lib_pk.so,build/variants/lib_lean.so \
  --modes pose_slerp,imu --rounds 8 > $OUT/ab.log 2>&1
rc=$?
tail -3 $OUT/tests.log; cat $OUT/ab.log
exit $rc
