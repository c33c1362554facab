set -u
OUT=gpurun_out/r3s08; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab.py --modes pose_slerp --replicas 3 --rounds 5 \
  --libs $V/lib_cur.so,$V/lib_slerpx.so,$V/lib_slerpnt.so,$V/lib_slerpxnt.so > $OUT/ab_slerp.log 2>&1 || exit $?
cp gpurun_out/ab.json $OUT/ab_slerp.json; grep replicas $OUT/ab_slerp.log
timeout -k 10 600 python -u tools/ab.py --modes imu,frame --replicas 3 --rounds 5 \
  --libs $V/lib_cur.so,$V/lib_d_sc1.so,$V/lib_d_nt.so,$V/lib_x_sc1.so > $OUT/ab_imu_frame.log 2>&1 || exit $?
cp gpurun_out/ab.json $OUT/ab_imu_frame.json; grep replicas $OUT/ab_imu_frame.log
timeout -k 10 600 python -u tools/ab_stager.py --replicas 2 \
  --libs $V/lib_su1.so,$V/lib_su2.so,$V/lib_su4.so,$V/lib_su2sc1.so,$V/lib_su1sc1.so,$V/lib_su2pl.so > $OUT/ab_stager.log 2>&1 || exit $?
tail -14 $OUT/ab_stager.log
timeout -k 10 600 python -u tools/pingpong.py --modes pose_slerp,imu --rounds 4 --steps 12 \
  --arms same,fread,fwrite,flush,f256,fslerp,fidle \
  --libs $PWD/livox-motion-compensation-sim_amd/libmcdeskew.so,$PWD/$V/lib_slerpx.so,$PWD/$V/lib_slerpnt.so \
  --out $OUT/pingpong.json > $OUT/pingpong.log 2>&1 || exit $?
cat $OUT/pingpong.log
