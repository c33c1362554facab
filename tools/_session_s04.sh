set -u
STEPS="tests ab" AB_ARGS="--replicas 3 --rounds 5" bash tools/gpu_session.sh s04 || exit $?
bash tools/sq_modes.sh s04/sq_f64c || exit $?
MCDESKEW_LIB=$PWD/build/variants/lib_r2f32.so bash tools/sq_modes.sh s04/sq_r2f32 || exit $?
