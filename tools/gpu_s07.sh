mkdir -p gpurun_out/r6s07
timeout -k 10 600 python -u bench.py > gpurun_out/r6s07/bench.json 2> gpurun_out/r6s07/bench.err
