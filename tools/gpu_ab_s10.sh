mkdir -p gpurun_out/r6s12
true && \
timeout -k 10 500 python -u tools/ab_pcd_fused.py --libs build/variants/lib_old.so,build/variants/lib_pk.so --modes pose_slerp,imu --rounds 10 > gpurun_out/r6s12/ab.log 2>&1
