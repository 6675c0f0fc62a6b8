"""Hydrate from the one-launch fields record, checked
on the CPU with the oracle's records and fields: BatchResult.Hydrate from
fields=True results without layouts fills every layer struct exactly as the
layouts path does (the HopByHop option map included), packet after packet,
reading no header on the host except where the record cannot describe the
stack. The device records are compared the same way in
test_hydrate_fields_gpu.py."""
import numpy as np

import hydrate_cases as H
import pktutil
from gopacket_amd import _lib
from gopacket_amd import gopacket as G
from gopacket_amd import layers as L


def _run(pkts, decoders=H.DECODERS, first=17, max_host=None):
    batch = G.PacketBatch.from_packets(pkts)
    pa, pb = H.parser(decoders, first), H.parser(decoders, first)
    ra, _, r = H.oracle_results(pa, batch, decoders)
    _, rb, _ = H.oracle_results(pb, batch, decoders)
    st = r["records"]["status"]
    idx = [i for i in range(len(pkts)) if (st[i] >> _lib.ST_NLAYERS_SHIFT & _lib.ST_NLAYERS_MASK) <= 16]
    n = H.compare(ra, rb, pa, pb, idx)
    if max_host is not None:
        assert rb.host_decodes <= max_host, rb.host_decodes
    return n, rb


def test_hbh_option_map_golden():
    """ip6_test.go:136-204 (TestPacketIPv6HopByHop0Decode): one PadN of 4
    bytes at HopByHop byte 2; the jumbogram header of ip6_test.go:349-432
    (TestIPv6JumbogramDecode): Jumbo Payload 0x00010008 at byte 2."""
    from oracle import oracle as O
    hop0 = pktutil.golden_bytes("ip6_hopbyhop0")
    jumbo = pktutil.golden_bytes("ip6_jumbogram_header") + b"\xfe" * 65536
    for pkt, want in ((hop0, [(1, 4, 6, bytes(4))]), (jumbo, [(0xC2, 4, 6, bytes([0, 1, 0, 8]))])):
        data, off, cap = pktutil.pack([pkt])
        r = O.OracleParser(21, ["IPV6", "IPV6_EXT", "PAYLOAD"]).decode(data, off, cap)
        f = O.extract_fields(data, off, r["layouts"]).view(_lib.FIELDS_DTYPE)[0]
        assert bytes(f["hbh_opt_map"]) == bytes([1, 0, 0])
        h = L.HopByHopFromMap(L.IPv6HopByHop(), pkt, 40, len(pkt), f["hbh_opt_map"])
        assert (h.NextHeader, h.HeaderLength, h.ActualLength) == (59, 0, 8)
        assert [(o.OptionType, o.OptionLength, o.ActualLength, o.OptionData) for o in h.Options] == want


def test_hydrate_fields_golden_and_hbh():
    pkts = [pktutil.golden_bytes(k) for k in ("simple_tcp", "vlan_tcp", "small_tcp_trailer", "udp_dns",
                                                "tcp_option_mss_eol", "mptcp_capable", "udp_too_small")]
    pkts += H.hbh_packets(1, 400)
    n, rb = _run(pkts)
    assert n == len(pkts)
    # only HopByHop headers past the map's 26 bytes (HeaderLength 3: a fifth of them) are read on the host
    assert 0 < rb.host_decodes < 400 * 0.35


def test_hydrate_fields_ipv6_raw_first():
    """ip6_test.go vectors decoded from LayerTypeIPv6 (LinkTypeRaw)."""
    pkts = [pktutil.golden_bytes("ip6_hopbyhop0"), pktutil.golden_bytes("ip6_destination0"),
            pktutil.golden_bytes("ip6_jumbogram_header") + b"\xfe" * 65536]
    n, rb = _run(pkts, decoders=(L.IPv6, L.IPv6ExtensionSkipper, L.UDP, L.TCP, G.Payload), first=21, max_host=0)
    assert n == 3


def test_hydrate_fields_fuzz():
    """Fuzzed packets (errors, truncation, tunnels, options, MPTCP, padding):
    identical structs; host reads only for the stacks the record cannot hold."""
    pkts = pktutil.fuzz_packets(5, 3000)
    n, rb = _run(pkts)
    assert n > 2900
    assert rb.host_decodes < 0.1 * n


def test_hydrate_fields_synthetic_c4_no_host_reads():
    """C4's IMIX mix (tags, QinQ, IPv6 with HopByHop): every packet from the
    record, none read on the host."""
    from gopacket_amd import synth
    pkts = [synth.packet(4, i) for i in range(5000)]
    n, rb = _run(pkts, max_host=0)
    assert n == 5000


def test_hydrate_fields_parser_subsets():
    """Parsers without some decoders (Unsupported / unknown next types end the
    list early): the slices still follow the decoded list."""
    pkts = pktutil.fuzz_packets(9, 800) + H.hbh_packets(2, 100)
    for decs in ((L.Ethernet, L.IPv4, L.TCP, G.Payload), (L.Ethernet, L.Dot1Q, L.IPv6, L.UDP),
                 (L.Ethernet, L.IPv4, L.IPv6, L.TCP, L.UDP, G.Fragment)):
        n, _ = _run(pkts, decoders=decs)
        assert n > 800


def test_ip_options_past_byte_255():
    """IPv4 and TCP headers starting past packet byte 254 (behind a 208-byte
    IPv6 Destination Options header: the record's one-byte starts read 0xFF):
    Hydrate and the option accessors derive the starts from the decoded list."""
    import struct
    ip = struct.pack(">BBHHHBBH4s4s", 0x46, 0, 24 + 28, 0, 0x4000, 64, 6, 0, bytes(4), bytes(4)) + bytes([7, 4, 4, 0])
    tcp = struct.pack(">HHIIBBHHH", 1, 2, 3, 4, 7 << 4, 0x12, 100, 0, 0) + bytes([2, 4, 5, 0xb4, 1, 1, 0, 0])
    dst = bytes([4, 25]) + bytes(206)  # NextHeader IPv4, (25 + 1) * 8 bytes
    ip6 = struct.pack(">IHBB16s16s", 0x60000000, len(dst) + len(ip) + len(tcp), 60, 64, bytes(16), bytes(16))
    pkt = bytes(12) + b"\x86\xdd" + ip6 + dst + ip + tcp
    n, rb = _run([pkt], max_host=0)
    assert n == 1
    batch = G.PacketBatch.from_packets([pkt])
    _, res, r = H.oracle_results(H.parser(), batch, H.DECODERS)
    assert int(r["records"][0]["status"]) & _lib.ST_ERR_MASK == 0
    assert int(res.fields[0]["ip4_start"]) == 0xFF and int(res.fields[0]["tcp_start"]) == 0xFF
    opts, pad = res.IPv4Options(0)
    assert [(o.OptionType, o.OptionLength) for o in opts] == [(7, 4)]
    opts, pad, mp = res.TCPOptions(0)
    assert [(o.OptionType, o.OptionLength) for o in opts] == [(2, 4), (1, 1), (1, 1), (0, 1)] and pad == b"\x00"
