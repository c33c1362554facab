set -u
OUT=gpurun_out/r3s45; mkdir -p $OUT
V=build/variants
for hz in 200 100 50 400; do
timeout -k 10 600 python -u tools/ab.py --modes imu,pose_slerp --replicas 2 --rounds 4 --imu-hz $hz --libs $V/lib_cur.so > $OUT/ab_imu_hz$hz.log 2>&1 || exit $?
echo "hz=$hz"; grep -E "replicas" $OUT/ab_imu_hz$hz.log
done
