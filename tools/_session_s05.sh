set -u
OUT=gpurun_out/s05; mkdir -p $OUT
STEPS="tests" bash tools/gpu_session.sh s05 || exit $?
V=build/variants
timeout -k 10 600 python -u tools/ab.py --modes frame --replicas 3 --rounds 5 \
  --libs $V/lib_r2f32.so,$V/lib_fq1.so,$V/lib_fq2.so,$V/lib_fq4.so,$V/lib_fsub.so > $OUT/ab_frame.log 2>&1 || exit $?
grep replicas $OUT/ab_frame.log
timeout -k 10 600 python -u tools/pingpong.py --modes pose_slerp,imu,frame --rounds 4 --steps 12 \
  --arms same,flush,fread,fwrite --libs $PWD/livox-motion-compensation-sim_amd/libmcdeskew.so,$PWD/$V/lib_slerpnt.so \
  --out $OUT/pingpong.json > $OUT/pingpong.log 2>&1 || exit $?
cat $OUT/pingpong.log
timeout -k 10 300 python -u tools/latency.py > $OUT/latency.json 2> $OUT/latency.err || exit $?
cat $OUT/latency.json
