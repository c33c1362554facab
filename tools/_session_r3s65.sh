set -u
OUT=gpurun_out/r3s65; mkdir -p $OUT
timeout -k 10 900 python tools/pmc_traffic.py --tag r3s65 > $OUT/pmc.log 2>&1 || exit $?
cut -c1-160 $OUT/pmc.log
timeout -k 10 600 python tools/pmc_traffic.py --aux --tag r3s65 > $OUT/pmc_aux.log 2>&1 || exit $?
cut -c1-160 $OUT/pmc_aux.log
