mkdir -p gpurun_out/r6s06
export MCDESKEW_ROWPIPE_TRACE=1
timeout -k 10 200 python -u tools/pin_probe.py > gpurun_out/r6s06/pin.json 2>&1 && \
timeout -k 10 400 python -u tools/host_path_probe.py --rows 1048576,2097152 --reps 4 > gpurun_out/r6s06/host_path.json 2> gpurun_out/r6s06/host_path.err && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_coords.py tests/test_gpu_scan.py > gpurun_out/r6s06/tests.log 2>&1
