#!/usr/bin/env python3
"""Fixtures for tests/c_abi (the C-language caller of include/gpk.h).

    python tools/make_c_abi_golden.py

Writes tests/golden/c_abi/:
  packets.bin  u32 count, then per packet: u32 caplen, caplen bytes
               (the golden packets of tests/golden: reference test vectors and
               the two reference capture files, plus 600 fuzzed packets)
  expect.bin   per parser configuration (statsassembly, eth_ip4_tcp_payload):
               n x gpk_record (16 B), n x 2 u32 err_args, 3n u64 flows (SoA)
  errors.txt   per configuration and packet with an error: "<cfg> <index> <Go error text>"
Expected values come from the oracle (oracle/, itself pinned to the
reference's vectors by tests/test_oracle_golden.py).
"""
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pktutil  # noqa: E402
from configs import CONFIGS, oracle_parser  # noqa: E402

CFGS = ("statsassembly", "eth_ip4_tcp_payload")


def packets():
    g = pktutil.golden()
    pk = [bytes.fromhex(v["hex"]) for k, v in sorted(g.items()) if "hex" in v]
    for name in ("test_ethernet.pcap", "test_dns.pcap"):
        pk += pktutil.read_pcap(os.path.join(pktutil.GOLDEN, name))[1]
    return pk + pktutil.fuzz_packets(2024, 600)


def main():
    out = os.path.join(ROOT, "tests", "golden", "c_abi")
    os.makedirs(out, exist_ok=True)
    pk = packets()
    with open(os.path.join(out, "packets.bin"), "wb") as f:
        f.write(struct.pack("<I", len(pk)))
        for p in pk:
            f.write(struct.pack("<I", len(p)) + p)
    data, off, cap = pktutil.pack(pk)
    lines = []
    with open(os.path.join(out, "expect.bin"), "wb") as f:
        for name in CFGS:
            op = oracle_parser(CONFIGS[name])
            r = op.decode(data, off, cap, layouts=False)
            f.write(r["records"].tobytes())
            f.write(r["err_args"].astype(np.uint32).tobytes())
            f.write(r["flows"].astype(np.uint64).tobytes())
            st = r["records"]["status"]
            for i in np.nonzero(st & 0x7F)[0]:
                code = int(st[i] & 0x7F)
                lines.append("%s %d %s" % (name, i, op.error_string(code, int(r["err_args"][2 * i]),
                                                                   int(r["err_args"][2 * i + 1]))))
    with open(os.path.join(out, "errors.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("%d packets, %d error lines" % (len(pk), len(lines)))


if __name__ == "__main__":
    main()
