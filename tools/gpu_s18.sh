mkdir -p gpurun_out/r6s18
export MCDESKEW_ROWPIPE_TRACE=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "alignment or align" > gpurun_out/r6s18/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/pcie_probe.py --mb 256 > gpurun_out/r6s18/pcie.json 2>&1 && \
timeout -k 10 300 python -u tools/host_path_probe.py --reps 5 > gpurun_out/r6s18/host_path.json 2> gpurun_out/r6s18/host_path.err
