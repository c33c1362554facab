mkdir -p gpurun_out/r6s14
true && \
timeout -k 10 500 python -u tools/ab_pcd_fused.py --libs build/variants/lib_pk0.so,build/variants/lib_pk1.so,build/variants/lib_pk2.so --modes pose_slerp,imu --rounds 8 > gpurun_out/r6s14/ab.log 2>&1
