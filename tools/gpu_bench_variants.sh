mkdir -p gpurun_out/r6s25
for args in "--mode imu" "--mode frame" "--issue calls" "--events-after"; do
  n=$(echo $args | tr -d ' -')
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu $args > gpurun_out/r6s25/$n.json 2> gpurun_out/r6s25/$n.err
  rc=$?
  echo "$args rc=$rc" >> gpurun_out/r6s25/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
