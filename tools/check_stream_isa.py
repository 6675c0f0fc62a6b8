#!/usr/bin/env python3
"""Build-time check of the dense phase-B stream's hand-scheduled loads.

The stream's loads are issued as inline asm (gpk_kernels.hip slot_load), so
the compiler's wait-count pass does not see them, and the kernel waits for
them itself (slot_wait). That is correct only if the compiled code leaves a
slot's registers alone while its load is in flight: a register copy, spill
or reuse of an in-flight register reads or clobbers stale data. The register
allocator is free to insert such copies (it believes the asm produced the
value at once), so every build is checked here instead of trusted.

Input: the device assembly of gpk_kernels.hip (hipcc -S --cuda-device-only,
same flags as the library). For every kernel, the instructions are walked in
layout order with the set of in-flight stream registers: an asm
buffer_load_dwordx4 ... nt puts its destination in flight; every later
vector-memory instruction ages it by one; s_waitcnt vmcnt(k) retires the
loads with at least k younger vector-memory operations behind them. Any
instruction that names an in-flight register is a violation.

    python tools/check_stream_isa.py kernels.s      exit 1 on a violation
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
VMEM = ("buffer_", "global_", "scratch_", "flat_")


def regs(operands):
    out = set()
    for m in REG.finditer(operands):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def check_function(name, lines):
    pending = []  # [regs, vmem ops issued after it, line number]
    in_asm = False
    bad = []
    nloads = 0
    for ln, raw in lines:
        line = raw.strip()
        if line.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if line.startswith(";;#ASMEND"):
            in_asm = False
            continue
        code = line.split(";")[0].strip()
        if not code or code.endswith(":") or code.startswith("."):
            continue
        mnem, _, ops = code.partition(" ")
        if mnem == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", ops)
            k = int(m.group(1)) if m else (0 if ops.strip() == "0" else None)
            if k is not None:
                pending = [p for p in pending if p[1] < k]
            continue
        used = regs(ops)
        for p in pending:
            if used & p[0]:
                bad.append("%s: line %d: '%s' touches v%s, in flight since line %d"
                           % (name, ln, code, sorted(used & p[0]), p[2]))
        if mnem.startswith(VMEM):
            for p in pending:
                p[1] += 1
            if in_asm and mnem == "buffer_load_dwordx4" and re.search(r"\bnt\b", ops):
                dst = ops.split(",")[0]
                pending.append([regs(dst), 0, ln])
                nloads += 1
    return bad, nloads


def main(path):
    text = open(path).read().split("\n")
    funcs, cur, start = {}, None, 0
    for i, l in enumerate(text):
        m = re.match(r"^(_Z\w*decode_kernel\w*):", l)
        if m:
            cur, start = m.group(1), i
        elif cur and l.startswith(".Lfunc_end"):
            funcs[cur] = [(k + 1, text[k]) for k in range(start, i)]
            cur = None
    if not funcs:
        print("check_stream_isa: no decode_kernel in %s" % path)
        return 1
    errors = 0
    for name, lines in funcs.items():
        bad, n = check_function(name, lines)
        for b in bad[:10]:
            print(b)
        errors += len(bad)
    print("check_stream_isa: %d kernels, %d violations" % (len(funcs), errors))
    return 1 if errors else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
