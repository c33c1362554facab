"""CPU sanitizer builds: the library's host-side code compiled with g++ under
AddressSanitizer + UndefinedBehaviorSanitizer and exercised here, no GPU needed.

* ``plan_host``: the batch layout / tile builder (``plan_batch``, behind ``mc_batch_create``) and
  the merged-cloud gather plan + its finishing copies (``plan_gather`` / ``gather_finish``, behind
  ``mc_comm_gather_batch`` and ``mc_gather_batches``) — ``csrc/plan.cpp`` itself, with host memcpy
  in place of the device copies and the RCCL receives; worlds 1-8, empty shards, 4/5-column
  shards, every root.
* ``pcd_formatter_host``: the device ``%.6f`` line writers (codecs.hpp), as in
  ``test_pcd_formatter_host.py``, now under the sanitizers.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "livox-motion-compensation-sim_amd", "csrc")
SAN = ["-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
       "-fno-omit-frame-pointer"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")

needs_gxx = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


@needs_gxx
def test_plan_host_under_asan_ubsan(tmp_path):
    exe = tmp_path / "plan_host"
    subprocess.run(["g++", *SAN, f"-I{CSRC}", os.path.join(ROOT, "tests", "host", "plan_host.cpp"),
                    os.path.join(CSRC, "plan.cpp"), "-o", str(exe)], check=True, capture_output=True, text=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "bad 0" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]


@needs_gxx
def test_pcd_formatter_under_asan_ubsan(tmp_path):
    from test_pcd_formatter_host import HARNESS, formatter_section
    code = open(HARNESS).read().replace("// FORMATTER_SECTION", formatter_section())
    cpp = tmp_path / "fmt.cpp"
    cpp.write_text(code)
    exe = tmp_path / "fmt"
    subprocess.run(["g++", *SAN, str(cpp), "-o", str(exe)],
                   check=True, capture_output=True, text=True)
    r = subprocess.run([str(exe), "50000"], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "bad 0" in r.stdout
    assert "runtime error" not in r.stderr, r.stderr[-3000:]
