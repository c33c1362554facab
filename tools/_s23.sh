L=build/variants/lib_base.so,build/variants/lib_new.so,build/variants/lib_new5.so
STEPS="tests abc abf pcdpmc" ABC_ARGS="--libs $L" ABF_ARGS="--libs $L --modes pose_slerp,frame" bash tools/gpu_session.sh r4s23 && \
timeout -k 10 600 python tools/pmc_traffic.py --aux --tag r4s23 > gpurun_out/r4s23/pmc_aux.log 2>&1 && cp profiles/pmc_traffic.json gpurun_out/r4s23/pmc_traffic.json && \
PMC_SET="TCC_HIT_sum TCC_MISS_sum SQ_WAVES" timeout -k 10 300 bash tools/pcd_pmc.sh > gpurun_out/r4s23/tcc.log 2>&1
