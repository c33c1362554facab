"""Kernel-by-kernel ISA comparison of two device assembly files (hipcc --cuda-device-only -S):
instructions only, comments and directives stripped.  For each kernel: same / DIFF (instruction
counts and the first differing pairs) / only in one file.

    python tools/isa_diff.py old.s new.s [--ignore-span]

--ignore-span drops the launch-span instructions (wall-clock stamps and their atomic / store) from
both sides before comparing, so a change confined to span_start / span_end reads as 'same*'.
"""
import re
import sys


def kernels(path):
    out, name, body = {}, None, []
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            name, body = m.group(1), []
            continue
        if name and line.startswith(".Lfunc_end"):
            out[name] = body
            name = None
            continue
        if name and line.startswith("\t") and not line.strip().startswith((".", ";")):
            # branch labels carry the function's index in the file (.LBB<fn>_<block>): drop it
            body.append(re.sub(r"\.LBB\d+_", ".LBB_", line.split(";")[0].rstrip()))
    return out


def strip_span(body):
    # the span code: s_memrealtime stamps and the stores / atomics that publish them
    return [l for l in body if "s_memrealtime" not in l and "global_atomic_umax_x2" not in l]


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    ign = "--ignore-span" in sys.argv
    for k in sorted(set(a) | set(b)):
        if k not in a or k not in b:
            print(f"only in {'new' if k in b else 'old'} {k}")
            continue
        x, y = a[k], b[k]
        if x == y:
            print(f"same {len(x)} {k}")
            continue
        if ign and strip_span(x) == strip_span(y):
            print(f"same* {len(x)} {len(y)} {k} (differs only in the launch-span code)")
            continue
        diffs = [(p, q) for p, q in zip(x, y) if p != q][:2]
        print(f"DIFF {len(x)} {len(y)} {k} {diffs}")


if __name__ == "__main__":
    main()
