#!/bin/bash
# GPU-box session for tuning: gpu tests, A/B of kernel variants, a 2-rank bench on one GPU
# (control plane + weak-scaling bookkeeping; RCCL refuses two ranks on one device, so the
# gather is expected to report an error there).  Stops at the first fault/abort/timeout.
set -u
TAG=${1:-ab}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
stop_if_fault() {
  echo "[$2] rc=$1" | tee -a "$OUT/steps_$TAG.log"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "[$2] fault/abort/timeout -> stopping"; exit "$1"; fi
}
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > "$OUT/pytest_gpu_$TAG.log" 2>&1
stop_if_fault $? pytest
tail -3 "$OUT/pytest_gpu_$TAG.log"

timeout -k 10 900 python tools/ab.py ${AB_ARGS:-} > "$OUT/ab_$TAG.log" 2>&1
stop_if_fault $? ab
cat "$OUT/ab_$TAG.log"

if [ "${SKIP_MULTI:-0}" = "0" ]; then
  MCDESKEW_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --no-extra-modes \
    > "$OUT/bench2_$TAG.json" 2> "$OUT/bench2_$TAG.err"
  stop_if_fault $? bench2
  cat "$OUT/bench2_$TAG.json"; tail -3 "$OUT/bench2_$TAG.err"
fi
