"""Inline-asm wide stores carry their own wait states (CPU; source and built-ISA checks).

A `global_store_dwordx4` reads its data VGPRs after issue; on gfx940+ a VALU write to them needs two
wait states after the store.  The compiler inserts them after its own stores but cannot see a
store inside inline asm, so every asm store of the library ends in `s_nop 1` (the
stager's `sc1` build lost the first 8 bytes of every 16-byte chunk without it).  The second test
reads the shipped library's gfx950 code objects: every sc1 store the kernels issue is followed by
`s_nop 1` (or more) before the next instruction.
"""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "livox-motion-compensation-sim_amd", "csrc")
LIB = os.path.join(ROOT, "livox-motion-compensation-sim_amd", "libmcdeskew.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

_ASM = re.compile(r'asm\s+volatile\s*\(\s*"([^"]*)"')


def _asm_stores():
    found = []
    for name in sorted(os.listdir(CSRC)):
        if not name.endswith((".hpp", ".hip", ".cpp")):
            continue
        with open(os.path.join(CSRC, name)) as f:
            for i, line in enumerate(f, 1):
                m = _ASM.search(line)
                if m and re.search(r"\b(global|buffer|flat)_store_dwordx[234]\b", m.group(1)):
                    found.append((name, i, m.group(1)))
    return found


def test_asm_stores_exist():
    # the deskew kernels' sc1 output stores are inline asm (kernels.hpp st_pol); if this fails the
    # check below checks nothing
    assert len(_asm_stores()) >= 1


def test_every_wide_asm_store_ends_in_two_wait_states():
    bad = []
    for name, line, text in _asm_stores():
        nop = re.search(r"s_nop\s+(\d+)\s*$", text.replace("\\n", "\n").replace("\\t", " ").strip())
        if not nop or int(nop.group(1)) < 1:
            bad.append(f"{name}:{line}: {text}")
    assert not bad, "asm stores without s_nop >= 1 after them:\n" + "\n".join(bad)


def test_built_library_sc1_stores_are_followed_by_wait_states(tmp_path):
    if not (os.path.exists(LIB) and os.path.exists(OBJDUMP)):
        pytest.skip("library not built or llvm-objdump missing")
    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)
    # --offloading writes the bundled code objects next to its input
    subprocess.run([OBJDUMP, "--offloading", str(lib)], cwd=tmp_path, check=True, capture_output=True)
    objs = glob.glob(str(tmp_path / "lib.so.*gfx950*"))
    assert objs, "no gfx950 code object in the library"
    stores, bad = 0, []
    for obj in objs:
        dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", obj], check=True, capture_output=True,
                             text=True).stdout.splitlines()
        ins = [ln.split("//")[0].strip() for ln in dis if ln.startswith("\t")]
        for i, s in enumerate(ins):
            # the asm form: sc1 alone (the compiler's own system-scope stores carry sc0 sc1 and get
            # their wait states from its hazard recognizer)
            if re.match(r"global_store_dwordx[234]\b.*\boff sc1$", s):
                stores += 1
                nxt = ins[i + 1] if i + 1 < len(ins) else ""
                m = re.match(r"s_nop\s+(\d+)", nxt)
                if not m or int(m.group(1)) < 1:
                    bad.append(f"{s}  ->  {nxt}")
    assert stores >= 3, f"expected the deskew kernels' sc1 stores in the ISA, found {stores}"
    assert not bad, "sc1 stores without two wait states behind them:\n" + "\n".join(bad)
