set -u
OUT=gpurun_out/r3s11; mkdir -p $OUT
V=build/variants
PYTEST_ARGS="-k codecs" STEPS="tests" bash tools/gpu_session.sh r3s11 || exit $?
timeout -k 10 600 python -u tools/ab_codecs.py --source batch --libs $V/lib_pww0.so,$V/lib_pww1.so > $OUT/ab_codecs.log 2>&1 || exit $?
tail -8 $OUT/ab_codecs.log
STEPS="bench" bash tools/gpu_session.sh r3s11 || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r3s11/bench.json'))
print(json.dumps(d['codecs']['pcd_ascii_fused'], indent=1)); print(d['codecs']['pcd_ascii']['frac'], d['codecs']['pcd_ascii']['kernels_ms'])"
