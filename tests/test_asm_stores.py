"""No vector-memory store hides inside inline asm (CPU; source check).

A `global_store_dwordx4` reads its data VGPRs after issue; on gfx940+ a VALU write to them needs two
wait states after the store.  The compiler's hazard recognizer inserts them only around stores it
can see.  Round 3 issued the sc1 output stores as inline asm with a hand-placed `s_nop 1` (the
stager's `sc1` build lost the first 8 bytes of every 16-byte chunk without it);
round 4 issues them through `__builtin_amdgcn_raw_buffer_store_b128` with the SC1 cache-policy bit
(kernels.hpp OutBuf), so the compiler owns the wait states and no asm store is left to audit.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "livox-motion-compensation-sim_amd", "csrc")

_ASM = re.compile(r'asm\s+(?:volatile\s*)?\(\s*"([^"]*)"')


def _sources():
    for name in sorted(os.listdir(CSRC)):
        if name.endswith((".hpp", ".hip", ".cpp")):
            with open(os.path.join(CSRC, name)) as f:
                yield name, f.read()


def test_no_vmem_store_in_inline_asm():
    bad = []
    for name, text in _sources():
        for i, line in enumerate(text.splitlines(), 1):
            m = _ASM.search(line)
            if m and re.search(r"\b(global|buffer|flat|scratch)_(store|atomic)", m.group(1)):
                bad.append(f"{name}:{i}: {m.group(1)}")
    assert not bad, "vector-memory stores inside inline asm:\n" + "\n".join(bad)


def test_sc1_output_stores_use_the_buffer_store_builtin():
    text = dict(_sources())["kernels.hpp"]
    assert "__builtin_amdgcn_raw_buffer_store_b128" in text
    assert re.search(r"constexpr int kBufSc1 = 16;", text)   # CPol::SC1 (= SCC) on gfx940+
    assert re.search(r"constexpr int kStorePol = 2;", text)
