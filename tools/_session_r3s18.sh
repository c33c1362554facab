set -u
OUT=gpurun_out/r3s18; mkdir -p $OUT
V=build/variants
timeout -k 10 900 python -u tools/ab.py --modes pose_slerp --replicas 2 --rounds 5 \
  --libs $V/lib_base.so,$V/lib_fuse.so,$V/lib_fusediag.so > $OUT/ab_fused_diag.log 2>&1 || exit $?
cp gpurun_out/ab.json $OUT/ab_fused_diag.json
grep -v replicas $OUT/ab_fused_diag.log | tail -6; grep replicas $OUT/ab_fused_diag.log
