set -u
OUT=gpurun_out/r3s15; mkdir -p $OUT
V=build/variants
timeout -k 10 900 python -u tools/ab.py --modes pose_slerp --replicas 2 --rounds 5 \
  --libs $V/lib_xspec.so,$V/lib_xnos.so,$V/lib_dspec.so,$V/lib_dnos.so,$V/lib_d2.so > $OUT/ab_slerp_fused.log 2>&1 || exit $?
cp gpurun_out/ab.json $OUT/ab_slerp_fused.json
grep -v replicas $OUT/ab_slerp_fused.log | tail -10; grep replicas $OUT/ab_slerp_fused.log
