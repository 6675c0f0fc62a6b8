"""The CPU oracle against the reference's own known-answer vectors.

Each test restates the expectation of the reference test it cites; the
packet bytes come from tests/golden/vectors.json (tools/harvest_golden.py).
Field values are read through the same host views (gopacket_amd.layers) the
product fills from device layouts; here the layouts come from the oracle.
"""
import struct

import numpy as np
import pytest

import pktutil
from oracle import oracle as O

ETH, D1Q, IP4, IP6, EXT, TCP, UDP, PAY = "ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP", "PAYLOAD"


def decode_one(first, decoders, pkt):
    p = O.OracleParser(first, decoders)
    data, off, cap = pktutil.pack([pkt])
    r = p.decode(data, off, cap)
    rec = r["records"][0]
    st = int(rec["status"])
    n = (st >> 8) & 0xFFF
    from gopacket_amd.engine import decode_codes
    return dict(rec=rec, st=st, decoded=decode_codes(rec["layers"], n), err=st & 0x7F,
                args=(int(r["err_args"][0]), int(r["err_args"][1])), trunc=bool(st & 0x80),
                flows=[int(x) for x in r["flows"]], layout=r["layouts"][0], parser=p, pkt=pkt)


def view(res, cls, slot):
    s, e = int(res["layout"]["start"][slot]), int(res["layout"]["end"][slot])
    assert s != 0xFFFFFFFF, "layer not decoded"
    v = cls()
    v._hydrate(res["pkt"][s:e])
    return v


# checksum_test.go:16-50
@pytest.mark.parametrize("name,want", [("cksum_two_carries", 0xfffe), ("cksum_wikipedia", 0xb861)])
def test_checksum_known_answers(name, want):
    b = bytearray(pktutil.golden_bytes(name))
    b[10] = b[11] = 0
    assert O.fold_checksum(O.compute_checksum(bytes(b))) == want


def test_fnv1a64_published_vectors():
    # flows.go:60-70 is FNV-1a 64; published vectors (no reference KAT exists)
    assert O.fnv_hash(b"") == 0xcbf29ce484222325
    assert O.fnv_hash(b"a") == 0xaf63dc4c8601ec8c
    assert O.fnv_hash(b"foobar") == 0x85944171f73967e8


def test_flow_fast_hash_symmetric():
    # flows.go:159-166: A->B and B->A collide
    a, b = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    assert O.flow_fast_hash(1, a, b) == O.flow_fast_hash(1, b, a)
    assert O.flow_fast_hash(1, a, b) != O.flow_fast_hash(2, a, b)


# layers/decode_test.go:386-492 TestDecodeSimpleTCPPacket + :1033-1043
def test_simple_tcp_packet():
    from gopacket_amd import layers
    r = decode_one(17, [ETH, IP4, TCP, PAY], pktutil.golden_bytes("simple_tcp"))
    assert r["decoded"] == [17, 20, 44, 2] and r["err"] == 0 and not r["trunc"]
    eth = view(r, layers.Ethernet, 0)
    assert eth.SrcMAC == bytes.fromhex("bc305be8d349") and eth.DstMAC == bytes.fromhex("00000c9ff020")
    ip = view(r, layers.IPv4, 2)
    assert (ip.Version, ip.IHL, ip.TOS, ip.Length, ip.Id, ip.Flags, ip.FragOffset, ip.TTL, ip.Protocol,
            ip.Checksum) == (4, 5, 0, 420, 14815, 2, 0, 64, 6, 0x555A)
    assert ip.SrcIP == bytes([172, 17, 81, 73]) and ip.DstIP == bytes([173, 222, 254, 225])
    assert ip.Contents == r["pkt"][14:34] and ip.Payload == r["pkt"][34:]
    tcp = view(r, layers.TCP, 5)
    assert (tcp.SrcPort, tcp.DstPort, tcp.Seq, tcp.Ack, tcp.DataOffset) == (50679, 80, 0xc57e0e48, 0x49074232, 8)
    assert tcp.ACK and tcp.PSH and not (tcp.FIN or tcp.SYN or tcp.RST or tcp.URG or tcp.ECE or tcp.CWR or tcp.NS)
    assert (tcp.Window, tcp.Checksum, tcp.Urgent) == (0x73, 0x9a8f, 0)
    assert [(o.OptionType, o.OptionLength, o.OptionData) for o in tcp.Options] == [
        (1, 1, None), (1, 1, None), (8, 10, bytes([0x3, 0x77, 0x37, 0x9c, 0x42, 0x77, 0x5e, 0x3a]))]
    assert tcp.Contents == r["pkt"][34:66] and tcp.Payload[:16] == b"GET / HTTP/1.1\r\n"
    # the packet's own checksums verify: Correct == Actual
    assert r["rec"]["ip4_csum"] == 0x555A and r["st"] & (1 << 21)
    assert r["rec"]["l4_csum"] == 0x9a8f and r["st"] & (1 << 23)
    # flow strings of the reference test: MAC, IP and port endpoints
    assert tcp.TransportFlow().String() == "50679->80"
    assert ip.NetworkFlow().String() == "172.17.81.73->173.222.254.225"
    assert eth.LinkFlow().String() == "bc:30:5b:e8:d3:49->00:00:0c:9f:f0:20"
    assert r["flows"] == [eth.LinkFlow().FastHash(), ip.NetworkFlow().FastHash(), tcp.TransportFlow().FastHash()]


# layers/decode_test.go:532-547: Ethernet trailer trimmed by IPv4 Length, TCP payload empty
def test_small_tcp_packet_has_empty_payload():
    r = decode_one(17, [ETH, IP4, TCP, PAY], pktutil.golden_bytes("small_tcp_trailer"))
    assert r["decoded"] == [17, 20, 44] and r["err"] == 0


# layers/decode_test.go:549-572 TestDecodeVLANPacket
def test_vlan_packet():
    r = decode_one(17, [ETH, D1Q, IP4, TCP, PAY], pktutil.golden_bytes("vlan_tcp"))
    assert r["decoded"][:4] == [17, 15, 20, 44] and r["err"] == 0


# layers/decode_test.go:1018-1031 TestDecodeUDPPacketTooSmall
def test_udp_packet_too_small_is_truncated():
    r = decode_one(17, [ETH, D1Q, IP4, UDP, PAY], pktutil.golden_bytes("udp_too_small"))
    assert r["decoded"] == [17, 15, 20, 45, 2] and r["trunc"] and r["err"] == 0


# layers/ip4_test.go:126-223 TestIPv4Options
@pytest.mark.parametrize("k,opts,padding", [
    (0, [(130, 11, bytes(9)), (0, 1, None)], None),
    (1, [(1, 1, None), (130, 11, bytes(9)), (0, 1, None)], bytes([1, 2, 3])),
    (2, [(130, 12, bytes(10))], None),
    (3, [(0, 1, None)], bytes([0x82, 0x0b] + [0] * 10 + [1, 2, 3])),
    (4, [(7, 7, bytes([4, 0, 0, 0, 0])), (1, 1, None), (0, 1, None)], bytes(3)),
])
def test_ipv4_options(k, opts, padding):
    from gopacket_amd import layers
    r = decode_one(20, [IP4], pktutil.golden_bytes("ip4_options_%d" % k))
    assert r["err"] in (0, 1)  # decodes (the next layer, ICMPv4, has no decoder)
    ip = view(r, layers.IPv4, 2)
    assert [(o.OptionType, o.OptionLength, o.OptionData) for o in ip.Options] == opts
    assert (ip.Padding or b"") == (padding or b"")  # bytes.Equal: nil == empty


# layers/ip4_test.go:102-113 TestIPv4InvalidOptionLength (option 136, length 0)
def test_ipv4_invalid_option_length():
    r = decode_one(20, [IP4], pktutil.golden_bytes("ip4_invalid_option_len"))
    assert r["err"] != 0 and r["decoded"] == []
    assert r["parser"].error_string(r["err"], *r["args"]) == "Invalid IP option type 136 length 0. Must be greater than 2"


# layers/tcp_test.go:87-109 TestPacketTCPOptionDecode: MSS 8192, EndList
def test_tcp_option_decode():
    from gopacket_amd import layers
    r = decode_one(17, [ETH, IP4, TCP, PAY], pktutil.golden_bytes("tcp_option_mss_eol"))
    assert r["err"] == 0
    tcp = view(r, layers.TCP, 5)
    assert [(o.OptionType, o.OptionLength, o.OptionData) for o in tcp.Options] == [(2, 4, bytes([32, 0])),
                                                                                   (0, 1, None)]


# layers/tcp_test.go:123-157 TestPacketMPTCPOptionDecode: MSS, MP_CAPABLE v1, EndList
def test_mptcp_option_decode():
    from gopacket_amd import layers
    r = decode_one(17, [ETH, IP4, TCP, PAY], pktutil.golden_bytes("mptcp_capable"))
    assert r["err"] == 0
    tcp = view(r, layers.TCP, 5)
    assert [(o.OptionType, o.OptionLength) for o in tcp.Options] == [(2, 4), (30, 4), (0, 1)]
    assert tcp.Options[1].OptionMultipath == 0 and tcp.Multipath


# layers/tcp_test.go:159-188 TestMPTCPInvalidLengthAndSubtype (the IPv4 packet after the SLL2 header)
def test_mptcp_bad_option_length():
    r = decode_one(20, [IP4, TCP, PAY], pktutil.golden_bytes("mptcp_bad_len_sll2")[20:])
    assert r["parser"].error_string(r["err"], *r["args"]).endswith("MPTCP bad option length 0")
    assert r["decoded"] == [20]


# layers/udp_test.go:39-98 TestUDPPacketDNS
def test_udp_packet_dns():
    from gopacket_amd import layers
    r = decode_one(17, [ETH, IP4, UDP, PAY], pktutil.golden_bytes("udp_dns"))
    assert r["decoded"] == [17, 20, 45]
    assert r["parser"].error_string(r["err"], *r["args"]) == "No decoder for layer type DNS"
    udp = view(r, layers.UDP, 6)
    assert (udp.SrcPort, udp.DstPort, udp.Length, udp.Checksum) == (53, 35181, 210, 30026)
    assert udp.Contents == bytes([0x0, 0x35, 0x89, 0x6d, 0x0, 0xd2, 0x75, 0x4a]) and len(udp.Payload) == 202


def _ip4_udp(src, dst, sport, dport, payload=b""):
    ip = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 28 + len(payload), 0, 0, 64, 17, 0, bytes(src), bytes(dst))
    return ip + struct.pack(">HHHH", sport, dport, 8 + len(payload), 0) + payload


# layers/tcpip_test.go:58-94 TestIPv4UDPChecksum: Wireshark 0xbc5f
def test_ipv4_udp_checksum():
    pkt = _ip4_udp([192, 0, 2, 1], [198, 51, 100, 1], 12345, 9999)
    r = decode_one(20, [IP4, UDP, PAY], pkt)
    assert r["decoded"] == [20, 45] and r["rec"]["l4_csum"] == 0xbc5f


# layers/tcpip_test.go:96-136 TestIPv6UDPChecksumWithIPv6DstOpts: Wireshark 0x4d21
def test_ipv6_dstopts_udp_checksum():
    src = bytes.fromhex("20010db8000000000000000000000001")
    dst = bytes.fromhex("20010db8000000000000000000000002")
    ext = bytes([17, 0, 0x01, 0x04, 0, 0, 0, 0])
    udp = struct.pack(">HHHH", 12345, 9999, 8, 0)
    ip6 = struct.pack(">IHBB16s16s", 0x60000000, len(ext) + len(udp), 60, 64, src, dst)
    r = decode_one(21, [IP6, EXT, UDP, PAY], ip6 + ext + udp)
    assert r["decoded"] == [21, 49, 45] and r["rec"]["l4_csum"] == 0x4d21


# layers/ip6_test.go:136-204 TestPacketIPv6HopByHop0Decode: Payload [] (and, per
# ip6.go:262-275, Truncated: the HopByHop bytes are counted twice)
def test_ipv6_hopbyhop0():
    from gopacket_amd import layers
    r = decode_one(21, [IP6, EXT, PAY], pktutil.golden_bytes("ip6_hopbyhop0"))
    assert r["decoded"] == [21] and r["err"] == 0 and r["trunc"]
    ip6 = view(r, layers.IPv6, 3)
    assert (ip6.Version, ip6.Length, ip6.NextHeader, ip6.HopLimit) == (6, 8, 0, 64)
    assert ip6.Payload == b"" and ip6.HopByHop.NextHeader == 59 and ip6.HopByHop.ActualLength == 8
    assert [(o.OptionType, o.OptionLength, o.ActualLength, o.OptionData) for o in ip6.HopByHop.Options] == [
        (1, 4, 6, bytes(4))]


# layers/ip6_test.go:246-304 TestPacketIPv6Destination0Decode
def test_ipv6_destination0():
    r = decode_one(21, [IP6, EXT, PAY], pktutil.golden_bytes("ip6_destination0"))
    assert r["decoded"] == [21, 49] and r["err"] == 0


# layers/ip6_test.go:349-432 TestIPv6JumbogramDecode: IPv6.Payload keeps the
# HopByHop header (ip6.go:249-256)
def test_ipv6_jumbogram():
    from gopacket_amd import layers
    pkt = pktutil.golden_bytes("ip6_jumbogram_header") + b"\xfe" * 65536
    r = decode_one(21, [IP6, PAY], pkt)
    assert r["decoded"] == [21, 2] and r["err"] == 0 and not r["trunc"]
    ip6 = view(r, layers.IPv6, 3)
    assert ip6.Length == 0 and ip6.Payload == pkt[40:]
    assert ip6.HopByHop.Options[0].OptionType == 0xC2 and ip6.HopByHop.Options[0].OptionData == bytes([0, 1, 0, 8])


# layers/tcpip_test.go:138-186 TestIPv6JumbogramUDPChecksum: ipv6UDPChecksumJumbogram
# = 0xcda8 (tcpip_test.go:19), the reference's one vector for a segment over 64 KiB
# and for the pseudo-header's length>>16 term (tcpip.go:54-69: 65544 bytes)
def test_ipv6_jumbogram_udp_checksum():
    pkt = pktutil.ipv6_udp_jumbogram()
    seg, src, dst = pkt[48:], pkt[8:24], pkt[24:40]
    assert len(seg) == 65544
    # computeChecksum (tcpip.go:54-69) as the oracle restates it: pseudo-header
    # addresses + protocol + length & 0xffff + length >> 16, then ComputeChecksum
    # over the segment mod 2^32 (checksum.go:35-50) and FoldChecksum
    csum = O.compute_checksum(src + dst) + 17 + (len(seg) & 0xFFFF) + (len(seg) >> 16)
    assert O.fold_checksum(O.compute_checksum(seg, csum)) == 0xcda8
    # the same through the oracle's decode: gopacket's test reads the layers of
    # NewPacket, where the HopByHop layer's payload feeds UDP; DecodingLayerParser
    # hands UDP the IPv6 Payload, which keeps the HopByHop header (ip6.go:249-256,
    # SURVEY P4): the UDP decoder sees Length 1 there and fails (udp.go:52-53)
    r = decode_one(21, [IP6, EXT, UDP, PAY], pkt)
    assert r["decoded"] == [21] and r["err"] == 61 and r["args"][0] == 1
    # a jumbogram whose IPv6 Payload is the UDP segment as DecodeLayers slices it:
    # a 16-byte HopByHop header (PadN, the Jumbo TLV at 4n+2, PadN) whose bytes 4-5
    # are 0, so the UDP decoder reads them as a jumbo Length 0 (udp.go:49-50)
    # and sums the whole rest of the packet, with length>>16 = 1
    pkt2 = pktutil.ipv6_udp_jumbogram(hbh16=True)
    r = decode_one(21, [IP6, EXT, UDP, PAY], pkt2)
    assert r["decoded"] == [21, 45, 2] and r["err"] == 0 and r["st"] & (1 << 22)
    seg2 = pkt2[40:]
    csum2 = O.compute_checksum(src + dst) + 17 + (len(seg2) & 0xFFFF) + (len(seg2) >> 16)
    existing = struct.unpack(">H", seg2[6:8])[0]
    assert r["rec"]["l4_csum"] == O.fold_checksum(O.compute_checksum(seg2, csum2) - existing)


# pcap/pcap_test.go:50-117: test_ethernet.pcap is 10 Eth/IPv4/TCP packets
def test_pcap_ethernet_fixture():
    link, pkts = pktutil.read_pcap(pktutil.GOLDEN + "/test_ethernet.pcap")
    assert link == 1 and len(pkts) == 10
    p = O.OracleParser(17, [ETH, IP4, TCP, PAY])
    data, off, cap = pktutil.pack(pkts)
    r = p.decode(data, off, cap)
    from gopacket_amd.engine import decode_codes
    st = r["records"]["status"]
    for i in range(10):
        lst = decode_codes(r["records"][i]["layers"], (int(st[i]) >> 8) & 0xFFF)
        assert lst[:3] == [17, 20, 44] and (st[i] & 0x7F) == 0
    assert np.all(st & (1 << 21)) and np.all(st & (1 << 23))  # every IPv4 and TCP checksum verifies
    # packets 0 and 1 run in opposite directions: identical symmetric flow hashes
    n = 10
    for k in range(3):
        assert r["flows"][k * n + 0] == r["flows"][k * n + 1]


def test_pcap_dns_fixture():
    link, pkts = pktutil.read_pcap(pktutil.GOLDEN + "/test_dns.pcap")
    assert len(pkts) == 10
    p = O.OracleParser(17, [ETH, IP4, UDP, PAY])
    data, off, cap = pktutil.pack(pkts)
    r = p.decode(data, off, cap)
    for i in range(10):
        assert p.error_string(int(r["records"][i]["status"] & 0x7F), *r["err_args"][2 * i:2 * i + 2]) == \
            "No decoder for layer type DNS"
