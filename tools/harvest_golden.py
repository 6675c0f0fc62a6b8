#!/usr/bin/env python3
"""Harvest the reference's own known-answer vectors for the hot path into
tests/golden/ (data only: packet bytes and the capture files the reference's
tests read).

Run in the build container, where /root/reference exists (read as text):

    python tools/harvest_golden.py /root/reference

Expected values (decoded layers, field values, checksums, error text) are NOT
harvested here: the tests in tests/test_oracle_golden.py restate them next to
the reference test that pins them (file:line), the way the reference's own
tests state them.
"""
import base64
import json
import os
import re
import sys

# name -> (file, line where the []byte{ literal starts (or a var name), kind)
ARRAYS = {
    # layers/decode_test.go:23-61 testSimpleTCPPacket (420 B Eth/IPv4/TCP HTTP GET)
    "simple_tcp": ("layers/decode_test.go", "testSimpleTCPPacket"),
    # layers/decode_test.go:532-547 TestDecodeSmallTCPPacketHasEmptyPayload (literal at :533)
    "small_tcp_trailer": ("layers/decode_test.go", 533),
    # layers/decode_test.go:549-572 TestDecodeVLANPacket
    "vlan_tcp": ("layers/decode_test.go", 551),
    # layers/decode_test.go:1018-1031 TestDecodeUDPPacketTooSmall
    "udp_too_small": ("layers/decode_test.go", 1019),
    # layers/tcp_test.go:80-86 / :116-122 / :161-167
    "tcp_option_mss_eol": ("layers/tcp_test.go", "testPacketTCPOptionDecode"),
    "mptcp_capable": ("layers/tcp_test.go", "testPacketMPTCPOptionDecode"),
    "mptcp_bad_len_sll2": ("layers/tcp_test.go", "testMPTCPInvalidLengthAndSubtype"),
    # layers/udp_test.go:36-53 testUDPPacketDNS
    "udp_dns": ("layers/udp_test.go", "testUDPPacketDNS"),
    # layers/ip6_test.go:96-100, :206-210, :306-310
    "ip6_hopbyhop0": ("layers/ip6_test.go", "testPacketIPv6HopByHop0"),
    "ip6_destination0": ("layers/ip6_test.go", "testPacketIPv6Destination0"),
    "ip6_jumbogram_header": ("layers/ip6_test.go", "testPacketIPv6JumbogramHeader"),
}

HEX = {
    # checksum_test.go:21-28
    "cksum_two_carries": ("checksum_test.go", r'"(4540005800000000ff11ffff0aeb1d070aed8877)"'),
    "cksum_wikipedia": ("checksum_test.go", r'"(45000073000040004011b861c0a80001c0a800c7)"'),
    # layers/ip4_test.go:104 TestIPv4InvalidOptionLength
    "ip4_invalid_option_len": ("layers/ip4_test.go", r'hex.DecodeString\("([0-9a-f]+)"\)'),
}

# layers/ip4_test.go:126-223 TestIPv4Options: the five packet strings
IP4_OPTIONS = ("layers/ip4_test.go", r'packet:\s*"([0-9a-f]+)"')

PCAPS = ["pcap/test_ethernet.pcap", "pcap/test_dns.pcap"]


def parse_array_at(text, start_idx):
    i = text.index("[]byte{", start_idx) + len("[]byte{")
    depth, j = 1, i
    while depth:
        if text[j] == "{":
            depth += 1
        elif text[j] == "}":
            depth -= 1
        j += 1
    body = text[i:j - 1]
    body = re.sub(r"//[^\n]*", "", body)
    return bytes(int(t, 0) for t in re.findall(r"0[xX][0-9a-fA-F]+|\d+", body))


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for name, (rel, loc) in ARRAYS.items():
        text = open(os.path.join(ref, rel)).read()
        if isinstance(loc, int):
            lines = text.split("\n")
            idx = len("\n".join(lines[:loc - 1]))
            data = parse_array_at(text, idx)
            src = "%s:%d" % (rel, loc)
        else:
            m = re.search(r"var %s = \[\]byte\{" % loc, text)
            data = parse_array_at(text, m.start())
            src = "%s:%d (%s)" % (rel, text[:m.start()].count("\n") + 1, loc)
        out[name] = {"source": src, "hex": data.hex()}
    for name, (rel, pat) in HEX.items():
        text = open(os.path.join(ref, rel)).read()
        m = re.search(pat, text)
        out[name] = {"source": "%s:%d" % (rel, text[:m.start()].count("\n") + 1), "hex": m.group(1)}
    rel, pat = IP4_OPTIONS
    text = open(os.path.join(ref, rel)).read()
    for k, m in enumerate(re.finditer(pat, text)):
        out["ip4_options_%d" % k] = {"source": "%s:%d" % (rel, text[:m.start()].count("\n") + 1),
                                     "hex": m.group(1)}
    for rel in PCAPS:
        raw = open(os.path.join(ref, rel), "rb").read()
        name = os.path.basename(rel)
        with open(os.path.join(repo, "tests", "golden", name), "wb") as f:
            f.write(raw)
        out[name] = {"source": rel, "file": name, "bytes": len(raw)}
    with open(os.path.join(repo, "tests", "golden", "vectors.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("harvested %d vectors" % len(out))


if __name__ == "__main__":
    main()
