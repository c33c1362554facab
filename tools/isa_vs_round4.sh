#!/bin/bash
# Device ISA of mcdeskew.hip: round 4's final commit (2fba479) vs this tree, kernel by kernel
# (tools/isa_diff.py).  Section A compiles this tree with round 4's span_end put back (the launch-span
# fold is the round's only intended deskew-kernel change), section B this tree as it is.
#   bash tools/isa_vs_round4.sh > profiles/round5/isa_diff_trim.txt
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d)
trap 'rm -rf "$W"' EXIT
HIPCC="${ROCM_PATH:-/opt/rocm}/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S"
mkdir -p "$W/r4" "$W/a" "$W/b"
git -C "$ROOT" archive 2fba479 livox-motion-compensation-sim_amd/csrc include | tar x -C "$W/r4"
for d in a b; do cp -r "$ROOT/livox-motion-compensation-sim_amd" "$ROOT/include" "$W/$d/"; done
python3 - "$W/a/livox-motion-compensation-sim_amd/csrc/kernels.hpp" <<'EOF'
import sys
p = sys.argv[1]; s = open(p).read()
a = s.index("__device__ __forceinline__ void span_end(unsigned long long* span) {")
b = s.index("\n}\n", a) + 3
s = s[:a] + """__device__ __forceinline__ void span_end(unsigned long long* span) {
  if (span && blockIdx.x + kSpanTail >= gridDim.x) {
    __syncthreads();
    const int k = (int)(blockIdx.x + kSpanTail - gridDim.x);
    if (threadIdx.x == 0) span[1 + k] = (unsigned long long)wall_clock64();
  }
}
""" + s[b:]
open(p, "w").write(s)
EOF
for d in r4 a b; do (cd "$W/$d/livox-motion-compensation-sim_amd/csrc" && $HIPCC mcdeskew.hip -o "$W/$d.s" 2>/dev/null); done
echo "Device ISA of mcdeskew.hip, round 4's final commit 2fba479 vs this tree ($(git -C "$ROOT" rev-parse --short HEAD)),"
echo "hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S, compared kernel by kernel by tools/isa_diff.py"
echo "(instructions only, branch-label function indices normalised).  Made by tools/isa_vs_round4.sh."
echo
echo "== A: this tree with round 4's span_end put back (the round's only deskew-kernel change is the span fold) =="
python3 "$ROOT/tools/isa_diff.py" "$W/r4.s" "$W/a.s"
echo
echo "== B: this tree as it is =="
python3 "$ROOT/tools/isa_diff.py" "$W/r4.s" "$W/b.s"
