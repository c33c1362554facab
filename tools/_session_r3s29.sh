set -u
OUT=gpurun_out/r3s29; mkdir -p $OUT
V=build/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -k "imu or IMU or compensate or steps or coherence" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_imu.log 2>&1 || exit $?
tail -2 $OUT/pytest_imu.log
timeout -k 10 900 python -u tools/ab.py --modes imu --replicas 4 --rounds 5 --check \
  --libs $V/lib_nt.so,$V/lib_sc1.so,$V/lib_sc1nt.so > $OUT/ab_imu_store.log 2>&1 || exit $?
grep -E "replicas|differ" $OUT/ab_imu_store.log
