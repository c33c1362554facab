set -u
OUT=gpurun_out/r3s25; mkdir -p $OUT
V=build/variants
timeout -k 10 900 python -u tools/ab.py --modes frame --replicas 2 --rounds 5 \
  --libs $V/lib_fu2.so,$V/lib_fu1.so,$V/lib_fu4.so,$V/lib_fnt.so,$V/lib_fsc1.so > $OUT/ab_frame.log 2>&1 || exit $?
grep replicas $OUT/ab_frame.log
