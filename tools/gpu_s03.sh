mkdir -p gpurun_out/r6s03
timeout -k 10 300 python -u tools/host_path_probe.py --variants 0,1,2,0,1,2 > gpurun_out/r6s03/host_path.json 2> gpurun_out/r6s03/host_path.err && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "alignment or known_answers or align" > gpurun_out/r6s03/tests.log 2>&1
