set -u
STEPS="tests" bash tools/gpu_session.sh r3s17 || exit $?
