mkdir -p gpurun_out/r6s10
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_codecs.py tests/test_gpu_scan.py tests/test_gpu_parity.py -k "pcd or stager or scan or aos" > gpurun_out/r6s10/tests.log 2>&1 && \
timeout -k 10 500 python -u tools/ab_pcd_fused.py --libs build/variants/lib_old.so,build/variants/lib_pk.so --modes pose_slerp,frame,imu --rounds 5 > gpurun_out/r6s10/ab.log 2>&1
