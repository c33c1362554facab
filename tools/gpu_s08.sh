mkdir -p gpurun_out/r6s08
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6s08/tests.log 2>&1
