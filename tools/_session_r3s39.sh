set -u
OUT=gpurun_out/r3s39; mkdir -p $OUT
timeout -k 10 1100 python -u tools/bench_configs.py --out $OUT/configs.json > $OUT/configs.log 2>&1 || exit $?
cut -c1-250 $OUT/configs.log
