mkdir -p gpurun_out/r6s02
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_scan.py tests/test_gpu_codecs.py tests/test_gpu_run.py > gpurun_out/r6s02/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/host_path_probe.py > gpurun_out/r6s02/host_path.json 2> gpurun_out/r6s02/host_path.err
