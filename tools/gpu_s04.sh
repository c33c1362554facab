mkdir -p gpurun_out/r6s04
export MCDESKEW_ROWPIPE_TRACE=1
timeout -k 10 400 python -u tools/host_path_probe.py --variants 0,1 --rows 262144,1048576,2097152 --reps 4 > gpurun_out/r6s04/host_path.json 2> gpurun_out/r6s04/host_path.err
