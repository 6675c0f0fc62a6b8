#!/usr/bin/env python3
"""Build-time check: the decode kernels the default launches select carry no
scratch (private segment) memory.

A kernel with `.private_segment_fixed_size` > 0 spills registers to scratch:
every spill and reload is a vector-memory round trip on the wave's latency
chain, and its dispatch needs a scratch allocation. The specialisations a
default launch can select (compact LDS tables, any output set, without and
with layouts, the stream-before-parse kernel and its fused-fields variant, the
fused grouping keys) must have none; the global-table kernels
(GPK_TABLES_GLOBAL, a test and diagnosis mode) are reported only.

Input: the device assembly of gpk_kernels.hip (hipcc -S --cuda-device-only,
same flags as the library; the Makefile runs this beside check_stream_isa.py).

    python tools/check_scratch.py kernels.s      exit 1 on scratch in a default kernel
"""
import re
import sys

# mangled template arguments: decode_kernel<kL4, kLayout, kCompact, ...>,
# decode_sb_kernel<kCompact, ...>
DECODE = re.compile(r"_ZN3gpk13decode_kernelILb([01])ELb([01])ELb([01])E")
SB = re.compile(r"_ZN3gpk16decode_sb_kernelILb([01])ELi\d+ELi\d+ELb([01])E")


# the fused decode + fields variant (decode_sb_kernel<..., kFields = true>) is
# held to the rule too, unless --lenient-fields (A/B builds of its budget)
STRICT_FIELDS = "--lenient-fields" not in sys.argv


def kernels(text):
    """(name, private segment bytes, VGPRs) of every kernel in the metadata."""
    out = []
    for b in text.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", b)
        priv = re.search(r"\.private_segment_fixed_size:\s+(\d+)", b)
        vg = re.search(r"\.vgpr_count:\s+(\d+)", b)
        if name and priv:
            out.append((name.group(1), int(priv.group(1)), int(vg.group(1)) if vg else -1))
    return out


def is_default(name):
    m = DECODE.match(name)
    if m:
        return m.group(3) == "1"
    m = SB.match(name)
    if m:
        return m.group(1) == "1" and (STRICT_FIELDS or m.group(2) == "0")
    return False


def main(path):
    ks = kernels(open(path).read())
    if not ks:
        print("check_scratch: no kernel metadata in %s" % path)
        return 1
    bad = 0
    n = 0
    for name, priv, vg in ks:
        if not (DECODE.match(name) or SB.match(name)):
            continue
        n += 1
        if priv and is_default(name):
            print("check_scratch: %s: %d bytes of scratch per lane (%d VGPRs)" % (name, priv, vg))
            bad += 1
        elif priv:
            print("check_scratch: (not checked: global tables) %s: %d bytes" % (name, priv))
    print("check_scratch: %d decode kernels, %d default kernels with scratch" % (n, bad))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main([x for x in sys.argv[1:] if not x.startswith("--")][0]))
