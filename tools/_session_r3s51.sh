set -u
bash tools/sq_modes.sh r3s51 || exit $?
