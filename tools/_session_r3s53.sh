set -u
OUT=gpurun_out/r3s53; mkdir -p $OUT
timeout -k 10 900 python tools/pmc_traffic.py --tag r3s53 > $OUT/pmc.log 2>&1 || exit $?
cat $OUT/pmc.log | cut -c1-300
timeout -k 10 600 python tools/pmc_traffic.py --aux --tag r3s53 > $OUT/pmc_aux.log 2>&1 || exit $?
cut -c1-200 $OUT/pmc_aux.log
timeout -k 10 1100 python -u tools/bench_configs.py --out $OUT/configs.json > $OUT/configs.log 2>&1 || exit $?
cut -c1-250 $OUT/configs.log
