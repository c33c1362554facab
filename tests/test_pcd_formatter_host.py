"""The device "%.6f" line writers (codecs.hpp: pcd_fast / pcd_fast_len / the packed and SWAR line
writers) compiled for the host with g++ and checked against the C library's correctly rounded
formatting — the kernel's own source, spliced into tests/host/pcd_formatter_host.cpp, exercised
on this CPU (no GPU): float32 / float64 values, exact ties, digit carries, -0.0, values near the
4294 cut-off, lanes of a tile written in reverse order into shared dwords."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODECS = os.path.join(ROOT, "livox-motion-compensation-sim_amd", "csrc", "codecs.hpp")
HARNESS = os.path.join(ROOT, "tests", "host", "pcd_formatter_host.cpp")


def formatter_section() -> str:
    src = open(CODECS).read()
    return src[src.index("struct PcdFast {"):src.index("constexpr int32_t kPcdSlowTile")]


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.parametrize("writer", ["bytes", "swar", "fields"])
def test_line_writers_match_printf(tmp_path, writer):
    swar = 0 if writer == "fields" else 1
    nbytes = 1 if writer == "bytes" else 0
    code = open(HARNESS).read().replace("// FORMATTER_SECTION", formatter_section())
    cpp = tmp_path / "fmt.cpp"
    cpp.write_text(code)
    exe = tmp_path / "fmt"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-DMC_PCD_SWAR={swar}", f"-DMC_PCD_BYTES={nbytes}", "-DMC_PCD_DIAG=0", str(cpp), "-o", str(exe)],
                   check=True, capture_output=True, text=True)
    r = subprocess.run([str(exe), "200000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "bad 0" in r.stdout
