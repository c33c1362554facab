"""Inline-asm wide stores carry their own wait states (CPU; source check).

A `global_store_dwordx4` reads its data VGPRs after issue; on gfx940+ a VALU write to them needs two
wait states after the store.  The compiler inserts them after its own stores but cannot see a
store inside inline asm, so every asm store of the library ends in `s_nop 1` (the
stager's `sc1` build lost the first 8 bytes of every 16-byte chunk without it).
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "livox-motion-compensation-sim_amd", "csrc")

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
    # the per-point kernels' store policies are inline asm (kernels.hpp st_pol); if this fails the
    # check below checks nothing
    assert len(_asm_stores()) >= 3


def test_every_wide_asm_store_ends_in_two_wait_states():
    bad = []
    for name, line, text in _asm_stores():
        nop = re.search(r"s_nop\s+(\d+)\s*$", text.replace("\\n", "\n").replace("\\t", " ").strip())
        if not nop or int(nop.group(1)) < 1:
            bad.append(f"{name}:{line}: {text}")
    assert not bad, "asm stores without s_nop >= 1 after them:\n" + "\n".join(bad)
