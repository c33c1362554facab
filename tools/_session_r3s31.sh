set -u
OUT=gpurun_out/r3s31; mkdir -p $OUT
V=build/variants
timeout -k 10 600 python -u tools/ab_stager.py --replicas 3 --libs $V/lib_st1.so,$V/lib_st2.so,$V/lib_st4.so > $OUT/ab_stager_st.log 2>&1; rc=$?
tail -4 $OUT/ab_stager_st.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
tail -2 $OUT/pytest_gpu.log
