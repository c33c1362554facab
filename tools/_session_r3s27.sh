set -u
OUT=gpurun_out/r3s27; mkdir -p $OUT
V=build/variants
timeout -k 10 900 python -u tools/ab.py --modes imu --replicas 3 --rounds 5 --check \
  --libs $V/lib_base.so,$V/lib_seg.so > $OUT/ab_imu_segrec.log 2>&1 || exit $?
grep -E "replicas|identical|differ" $OUT/ab_imu_segrec.log
