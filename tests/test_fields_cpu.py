"""Layer fields (include/gpk.h gpk_fields): the oracle's field extraction
(oracle/gpk_oracle.c oracle_extract_fields) against the field values the
reference's own tests expect, and the record layout the C ABI declares.

Each test cites the reference test whose expectations it restates; the packet
bytes come from tests/golden/vectors.json (tools/harvest_golden.py).
"""
import struct

import numpy as np

import pktutil
from gopacket_amd import _lib
from oracle import oracle as O

ETH, D1Q, IP4, IP6, EXT, TCP, UDP, PAY = "ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP", "PAYLOAD"


def fields_of(first, decoders, pkts):
    p = O.OracleParser(first, decoders)
    data, off, cap = pktutil.pack(pkts)
    r = p.decode(data, off, cap)
    raw = O.extract_fields(data, off, r["layouts"])
    return raw.view(_lib.FIELDS_DTYPE).reshape(-1), r


def test_fields_record_layout():
    assert _lib.FIELDS_DTYPE.itemsize == 128
    for name, off in (("present", 0), ("hbh_opt_map", 1), ("eth_type", 4), ("eth_dst", 8), ("d1q_tci", 20), ("ip4_length", 28), ("ip6_flow_label", 40),
                      ("ip4_src", 48), ("ip6_src", 56), ("ip6_dst", 72), ("tcp_seq", 92), ("tcp_flags", 100),
                      ("udp_checksum", 114), ("ip4_start", 116), ("tcp_start", 117), ("ip4_opt_map", 118),
                      ("tcp_opt_map", 123)):
        assert _lib.FIELDS_DTYPE.fields[name][1] == off, name


# layers/decode_test.go:386-460 TestDecodeSimpleTCPPacket
def test_simple_tcp_fields():
    f, _ = fields_of(17, [ETH, IP4, TCP, PAY], [pktutil.golden_bytes("simple_tcp")])
    f = f[0]
    assert int(f["present"]) == 0b10100101  # Ethernet, IPv4, TCP, Payload
    assert bytes(f["eth_src"]) == bytes.fromhex("bc305be8d349") and bytes(f["eth_dst"]) == bytes.fromhex("00000c9ff020")
    assert int(f["eth_type"]) == 0x0800 and int(f["eth_length"]) == 0
    assert (int(f["ip4_version"]), int(f["ip4_ihl"]), int(f["ip4_tos"]), int(f["ip4_length"]), int(f["ip4_id"]),
            int(f["ip4_flags_frag"]) >> 13, int(f["ip4_flags_frag"]) & 0x1FFF, int(f["ip4_ttl"]),
            int(f["ip4_protocol"]), int(f["ip4_checksum"])) == (4, 5, 0, 420, 14815, 2, 0, 64, 6, 0x555A)
    assert bytes(f["ip4_src"]) == bytes([172, 17, 81, 73]) and bytes(f["ip4_dst"]) == bytes([173, 222, 254, 225])
    assert (int(f["tcp_src_port"]), int(f["tcp_dst_port"]), int(f["tcp_seq"]), int(f["tcp_ack"]),
            int(f["tcp_data_offset"])) == (50679, 80, 0xc57e0e48, 0x49074232, 8)
    B = _lib.TCP_FLAG_BITS
    assert int(f["tcp_flags"]) == B["ACK"] | B["PSH"]
    assert (int(f["tcp_window"]), int(f["tcp_checksum"]), int(f["tcp_urgent"])) == (0x73, 0x9a8f, 0)
    # absent layers read 0
    assert int(f["udp_length"]) == 0 and int(f["ip6_version"]) == 0
    # option maps: no IPv4 options; TCP NOP, NOP, Timestamps at header bytes 20, 21, 22
    assert (int(f["ip4_start"]), int(f["tcp_start"])) == (14, 34)
    assert bytes(f["ip4_opt_map"]) == bytes(5) and bytes(f["tcp_opt_map"]) == bytes([0b111, 0, 0, 0, 0])


# layers/udp_test.go:39-98 TestUDPPacketDNS
def test_udp_dns_fields():
    f, _ = fields_of(17, [ETH, IP4, UDP, PAY], [pktutil.golden_bytes("udp_dns")])
    f = f[0]
    assert (int(f["udp_src_port"]), int(f["udp_dst_port"]), int(f["udp_length"]), int(f["udp_checksum"])) == \
        (53, 35181, 210, 30026)


# layers/ip6_test.go:136-160 TestPacketIPv6HopByHop0Decode
def test_ipv6_hopbyhop0_fields():
    f, _ = fields_of(21, [IP6, EXT, PAY], [pktutil.golden_bytes("ip6_hopbyhop0")])
    f = f[0]
    assert (int(f["ip6_version"]), int(f["ip6_traffic_class"]), int(f["ip6_flow_label"]), int(f["ip6_length"]),
            int(f["ip6_next_header"]), int(f["ip6_hop_limit"])) == (6, 0, 0, 8, 0, 64)
    assert bytes(f["ip6_src"]) == bytes.fromhex("20010db8000000000000000000000001")
    assert bytes(f["ip6_dst"]) == bytes.fromhex("20010db8000000000000000000000002")


# layers/dot1q_test.go:43-60 TestEncodeDecodeDot1Q: {Priority 3, VLAN 30} and
# {Priority 7, DropEligible, VLAN 0xFFF}, as dot1q.go:60-75 serializes them
def test_dot1q_fields():
    pkts = []
    for prio, de, vid in ((3, 0, 30), (7, 1, 0xFFF)):
        tci = prio << 13 | de << 12 | vid
        pkts.append(bytes(6) + bytes([2, 0, 0, 0, 0, 1]) + struct.pack(">HHH", 0x8100, tci, 0x0800) + bytes(20))
    f, _ = fields_of(17, [ETH, D1Q], pkts)
    got = [(int(x["d1q_tci"]) >> 13, int(x["d1q_tci"]) >> 12 & 1, int(x["d1q_tci"]) & 0xFFF, int(x["d1q_type"]))
           for x in f]
    assert got == [(3, 0, 30, 0x0800), (7, 1, 0xFFF, 0x0800)]


# layers/ethernet.go:50-55: an 802.3 length field, EthernetTypeLLC (enums.go:36)
def test_ethernet_llc_length():
    pkt = bytes(6) + bytes([2, 0, 0, 0, 0, 1]) + struct.pack(">H", 46) + bytes(46)
    f, _ = fields_of(17, [ETH], [pkt])
    assert int(f[0]["eth_type"]) == 0 and int(f[0]["eth_length"]) == 46


# layers/ip4.go:189-194: IPv4 Length 0 (TSO) reads as the slice's length
def test_ipv4_tso_length():
    ip = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 0, 7, 0x4000, 64, 6, 0, bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2]))
    tcp = struct.pack(">HHIIBBHHH", 1, 2, 3, 4, 5 << 4, 0x12, 100, 0, 0)
    f, _ = fields_of(20, [IP4, TCP, PAY], [ip + tcp + b"xyz"])
    assert int(f[0]["ip4_length"]) == 20 + 20 + 3 and int(f[0]["ip4_flags_frag"]) == 0x4000
    assert int(f[0]["tcp_flags"]) == 0x12 and int(f[0]["tcp_data_offset"]) == 5


def test_fields_match_hydrated_layers():
    """Fuzzed and synthetic packets: every field equals the gopacket-shaped layer
    struct (gopacket_amd.layers) filled from the same oracle layout."""
    from gopacket_amd import layers
    pkts = list(pktutil.fuzz_packets(7, 400))
    from gopacket_amd import synth
    pkts += [synth.packet(4, i) for i in range(300)] + [pktutil.golden_bytes("simple_tcp"),
                                                        pktutil.golden_bytes("vlan_tcp")]
    f, r = fields_of(17, [ETH, D1Q, IP4, IP6, EXT, TCP, UDP, PAY], pkts)
    checked = 0
    for i, pkt in enumerate(pkts):
        lay = r["layouts"][i]
        for slot, cls in ((0, layers.Ethernet), (2, layers.IPv4), (3, layers.IPv6), (5, layers.TCP), (6, layers.UDP)):
            s, e = int(lay["start"][slot]), int(lay["end"][slot])
            if s == _lib.LAYOUT_ABSENT:
                continue
            v = cls()
            v._hydrate(pkt[s:e])
            x = f[i]
            if cls is layers.Ethernet:
                assert (bytes(x["eth_src"]), bytes(x["eth_dst"]), int(x["eth_type"]), int(x["eth_length"])) == \
                    (bytes(v.SrcMAC), bytes(v.DstMAC), int(v.EthernetType), int(v.Length))
            elif cls is layers.IPv4:
                assert (int(x["ip4_ttl"]), int(x["ip4_length"]), int(x["ip4_id"]), bytes(x["ip4_src"])) == \
                    (v.TTL, v.Length, v.Id, bytes(v.SrcIP))
            elif cls is layers.IPv6:
                assert (int(x["ip6_flow_label"]), int(x["ip6_length"]), int(x["ip6_hop_limit"]),
                        bytes(x["ip6_dst"])) == (v.FlowLabel, v.Length, v.HopLimit, bytes(v.DstIP))
            elif cls is layers.TCP:
                assert (int(x["tcp_seq"]), int(x["tcp_ack"]), int(x["tcp_window"]), int(x["tcp_src_port"])) == \
                    (v.Seq, v.Ack, v.Window, int(v.SrcPort))
            else:
                assert (int(x["udp_length"]), int(x["udp_dst_port"])) == (v.Length, int(v.DstPort))
            checked += 1
    assert checked > 600


def options_of(f, pkt, r, i, cls):
    from gopacket_amd import layers
    if cls == "ip4":
        return layers.IPv4OptionsFromMap(pkt, int(f["ip4_start"]), int(f["ip4_ihl"]) * 4, f["ip4_opt_map"])
    return layers.TCPOptionsFromMap(pkt, int(f["tcp_start"]), int(f["tcp_data_offset"]) * 4, f["tcp_opt_map"])


# layers/ip4_test.go:126-223 TestIPv4Options: the option lists and Padding the
# reference expects, from the option maps alone
def test_ipv4_option_maps():
    want = {0: ([(130, 11, bytes(9)), (0, 1, None)], None),
            1: ([(1, 1, None), (130, 11, bytes(9)), (0, 1, None)], bytes([1, 2, 3])),
            2: ([(130, 12, bytes(10))], None),
            3: ([(0, 1, None)], bytes([0x82, 0x0b] + [0] * 10 + [1, 2, 3])),
            4: ([(7, 7, bytes([4, 0, 0, 0, 0])), (1, 1, None), (0, 1, None)], bytes(3))}
    for k, (opts, padding) in want.items():
        pkt = pktutil.golden_bytes("ip4_options_%d" % k)
        f, r = fields_of(20, [IP4], [pkt])
        assert int(f[0]["ip4_start"]) == 0
        got, pad = options_of(f[0], pkt, r, 0, "ip4")
        assert [(o.OptionType, o.OptionLength, o.OptionData) for o in got] == opts, k
        assert (pad or b"") == (padding or b""), k


# layers/tcp_test.go:87-109 (MSS 8192, EndList) and :123-157 (MSS, MP_CAPABLE v1, EndList)
def test_tcp_option_maps():
    pkt = pktutil.golden_bytes("tcp_option_mss_eol")
    f, r = fields_of(17, [ETH, IP4, TCP, PAY], [pkt])
    got, pad, mp = options_of(f[0], pkt, r, 0, "tcp")
    assert [(o.OptionType, o.OptionLength, o.OptionData) for o in got] == [(2, 4, bytes([32, 0])), (0, 1, None)]
    assert not mp
    pkt = pktutil.golden_bytes("mptcp_capable")
    f, r = fields_of(17, [ETH, IP4, TCP, PAY], [pkt])
    got, pad, mp = options_of(f[0], pkt, r, 0, "tcp")
    assert [(o.OptionType, o.OptionLength) for o in got] == [(2, 4), (30, 4), (0, 1)]
    assert got[1].OptionMultipath == 0 and mp


def test_option_maps_match_hydrated_layers():
    """Fuzzed packets (IPv4 options, TCP options incl. MPTCP and bad lengths):
    the lists rebuilt from the option maps equal the lists the layer structs
    decode from the same slices, Padding and Multipath included."""
    from gopacket_amd import layers
    from gopacket_amd import synth
    pkts = list(pktutil.fuzz_packets(11, 3000)) + [pktutil.golden_bytes("simple_tcp")]
    pkts += [synth.packet(4, i) for i in range(50)]
    # Linux SYN options, SACK blocks, EOL with padding, an MPTCP option
    for opts in (bytes([2, 4, 5, 0xb4, 4, 2, 8, 10]) + bytes(8) + bytes([1, 3, 3, 7]),
                 bytes([1, 1, 5, 18]) + bytes(16) + bytes([1, 1, 8, 10]) + bytes(8),
                 bytes([2, 4, 1, 0, 0, 9, 9, 9]), bytes([30, 4, 0x10, 0, 1, 0, 0, 0])):
        ip = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 40 + len(opts), 0, 0, 64, 6, 0, bytes(4), bytes(4))
        tcp = struct.pack(">HHIIBBHHH", 1, 2, 3, 4, (5 + len(opts) // 4) << 4, 0x12, 100, 0, 0) + opts
        pkts.append(bytes(12) + b"\x08\x00" + ip + tcp)
    f, r = fields_of(17, [ETH, D1Q, IP4, IP6, EXT, TCP, UDP, PAY], pkts)
    n4 = nt = 0
    for i, pkt in enumerate(pkts):
        lay = r["layouts"][i]
        s = int(lay["start"][2])
        if s != _lib.LAYOUT_ABSENT and s < 0xFF:
            v = layers.IPv4()
            v._hydrate(pkt[s:int(lay["end"][2])])
            got, pad = options_of(f[i], pkt, r, i, "ip4")
            assert got == v.Options and (pad or b"") == (v.Padding or b""), i
            n4 += len(got) > 0
        s = int(lay["start"][5])
        if s != _lib.LAYOUT_ABSENT and s < 0xFF:
            v = layers.TCP()
            v._hydrate(pkt[s:int(lay["end"][5])])
            got, pad, mp = options_of(f[i], pkt, r, i, "tcp")
            assert got == v.Options and pad == v.Padding and mp == v.Multipath, i
            nt += len(got) > 0
    assert n4 > 20 and nt > 25
