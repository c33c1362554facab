set -u
STEPS="tests smoke bench" bash tools/gpu_session.sh r3s10 || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r3s10/bench.json'))
print(json.dumps(d['codecs']['pcd_ascii_fused'], indent=1)); print(d['codecs']['pcd_ascii']['frac'])"
