"""The gopacket-shaped Python API (gopacket_amd.gopacket / .layers) on the GPU.

These read like the reference's own DecodingLayerParser tests: build a
parser from layer structs, DecodeLayers a packet, check `decoded`, the error,
Truncated, the layer fields, VerifyChecksum and the flows. Every call goes
through the HIP kernels (C ABI); expectations restate the cited reference
tests.
"""
import struct

import numpy as np
import pytest

import pktutil

pytestmark = pytest.mark.gpu


@pytest.fixture()
def gp(gpu_ctx):
    from gopacket_amd import gopacket, layers
    return gopacket, layers, gpu_ctx


def _parser(gp, first, *decs):
    gopacket, layers, ctx = gp
    return gopacket.DecodingLayerParser(first, *decs, ctx=ctx)


# layers/decode_test.go:386-492 TestDecodeSimpleTCPPacket through the parser
# (the DecodingLayerParser form of decode_test.go:192-205)
def test_decode_layers_simple_tcp(gp):
    gopacket, L, _ = gp
    eth, ip4, tcp, pay = L.Ethernet(), L.IPv4(), L.TCP(), gopacket.Payload()
    p = _parser(gp, L.LayerTypeEthernet, eth, ip4, tcp, pay)
    decoded = [L.LayerTypeDot1Q]  # truncated by DecodeLayers
    pkt = pktutil.golden_bytes("simple_tcp")
    err = p.DecodeLayers(pkt, decoded)
    assert err is None and not p.Truncated
    assert decoded == [L.LayerTypeEthernet, L.LayerTypeIPv4, L.LayerTypeTCP, gopacket.LayerTypePayload]
    assert eth.SrcMAC == bytes.fromhex("bc305be8d349") and eth.EthernetType == 0x0800
    assert (ip4.Length, ip4.Id, ip4.TTL, ip4.Protocol) == (420, 14815, 64, 6)
    assert (tcp.SrcPort, tcp.DstPort, tcp.Seq) == (50679, 80, 0xc57e0e48)
    assert pay.Payload() == pkt[66:]
    e, res = ip4.VerifyChecksum()
    assert e is None and res.Valid and res.Correct == res.Actual == 0x555A
    e, res = tcp.VerifyChecksum()
    assert e is None and res.Valid and res.Correct == 0x9a8f
    assert tcp.TransportFlow().String() == "50679->80"
    assert ip4.NetworkFlow().FastHash() == ip4.NetworkFlow().Reverse().FastHash()


# layers/decode_test.go:549-572 TestDecodeVLANPacket
def test_decode_layers_vlan(gp):
    gopacket, L, _ = gp
    eth, d1q, ip4, tcp, pay = L.Ethernet(), L.Dot1Q(), L.IPv4(), L.TCP(), gopacket.Payload()
    p = _parser(gp, L.LayerTypeEthernet, eth, d1q, ip4, tcp, pay)
    decoded = []
    err = p.DecodeLayers(pktutil.golden_bytes("vlan_tcp"), decoded)
    assert err is None
    assert decoded[:4] == [L.LayerTypeEthernet, L.LayerTypeDot1Q, L.LayerTypeIPv4, L.LayerTypeTCP]
    assert d1q.Type == 0x0800


# layers/udp_test.go:39-98 TestUDPPacketDNS: DNS has no decoder -> UnsupportedLayerType
def test_unsupported_layer_type_error(gp):
    gopacket, L, _ = gp
    p = _parser(gp, L.LayerTypeEthernet, L.Ethernet(), L.IPv4(), L.UDP(), gopacket.Payload())
    decoded = []
    err = p.DecodeLayers(pktutil.golden_bytes("udp_dns"), decoded)
    assert isinstance(err, gopacket.UnsupportedLayerType)
    assert err.Error() == "No decoder for layer type DNS"
    assert decoded == [L.LayerTypeEthernet, L.LayerTypeIPv4, L.LayerTypeUDP]
    p.IgnoreUnsupported = True
    assert p.DecodeLayers(pktutil.golden_bytes("udp_dns"), decoded) is None


# layers/decode_test.go:1018-1031 TestDecodeUDPPacketTooSmall: truncated, no error
def test_truncated_flag(gp):
    gopacket, L, _ = gp
    p = _parser(gp, L.LayerTypeEthernet, L.Ethernet(), L.Dot1Q(), L.IPv4(), L.UDP(), gopacket.Payload())
    decoded = []
    assert p.DecodeLayers(pktutil.golden_bytes("udp_too_small"), decoded) is None
    assert p.Truncated


# layers/tcp_test.go:159-188 TestMPTCPInvalidLengthAndSubtype: decoder error text
def test_decoder_error_text(gp):
    gopacket, L, _ = gp
    p = _parser(gp, L.LayerTypeIPv4, L.IPv4(), L.TCP(), gopacket.Payload())
    decoded = []
    err = p.DecodeLayers(pktutil.golden_bytes("mptcp_bad_len_sll2")[20:], decoded)
    assert err is not None and err.Error().endswith("MPTCP bad option length 0")
    assert decoded == [L.LayerTypeIPv4]


# parser.go:329-333: a short MPTCP option panics in Go; DecodeLayers returns
# "panic: runtime error: ..." unless IgnorePanic, which re-raises
def test_mptcp_panic_error(gp):
    gopacket, L, _ = gp
    ip = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + 24, 0, 0, 64, 6, 0, b"\x01" * 4, b"\x02" * 4)
    # MPTCP ADD_ADDR (subtype 4) claiming 5 bytes in a 4-byte option area: data[4] (tcp.go:414-455)
    tcp = struct.pack(">HHIIBBHHH", 1, 2, 0, 0, 0x60, 0x10, 0, 0, 0) + bytes([30, 5, 0x40, 0])
    p = _parser(gp, L.LayerTypeIPv4, L.IPv4(), L.TCP(), gopacket.Payload())
    decoded = []
    err = p.DecodeLayers(ip + tcp, decoded)
    assert err is not None and err.Error() == "panic: runtime error: index out of range [4] with length 4"
    p.IgnorePanic = True
    with pytest.raises(gopacket.GoPanic):
        p.DecodeLayers(ip + tcp, decoded)


# pcap/pcap_test.go:50-117 + the doc.go:211-228 batch pattern: DecodeBatch over
# test_ethernet.pcap, per-packet views agree with per-packet DecodeLayers
def test_decode_batch_matches_decode_layers(gp):
    gopacket, L, _ = gp
    _, pkts = pktutil.read_pcap(pktutil.GOLDEN + "/test_ethernet.pcap")
    eth, ip4, tcp, pay = L.Ethernet(), L.IPv4(), L.TCP(), gopacket.Payload()
    p = _parser(gp, L.LayerTypeEthernet, eth, ip4, tcp, pay)
    res = p.DecodeBatch(gopacket.PacketBatch.from_packets(pkts), layouts=True)
    assert len(res) == 10
    for i, pkt in enumerate(pkts):
        d1, d2 = [], []
        assert res.Hydrate(i, d1) is None
        h = res.FlowHashes(i)
        assert p.DecodeLayers(pkt, d2) is None
        assert d1 == d2 and d1[:3] == [L.LayerTypeEthernet, L.LayerTypeIPv4, L.LayerTypeTCP]
        assert res.IPv4Checksum(i)[0] and res.L4Checksum(i)[0]
        assert h == (eth.LinkFlow().FastHash(), ip4.NetworkFlow().FastHash(), tcp.TransportFlow().FastHash())
    assert res.FlowHashes(0) == res.FlowHashes(1)  # opposite directions, symmetric hash
    assert np.count_nonzero([gopacket.LayerTypePayload in res.Decoded(i) for i in range(10)]) == 3


# layers/decode_test.go:1045-1077 testDecodingLayerContainer over Map / Sparse / Array,
# and decode_test.go:1033-1043 TestDecodingLayerParserFullTCPPacket
@pytest.mark.parametrize("form", ["DecodingLayerMap", "DecodingLayerSparse", "DecodingLayerArray"])
def test_decoding_layer_container(gp, form):
    gopacket, L, ctx = gp
    dlc = getattr(gopacket, form)(None)
    dlc = dlc.Put(L.Ethernet())
    dlc = dlc.Put(L.IPv4())
    dlc = dlc.Put(L.TCP())
    dlc = dlc.Put(gopacket.Payload())
    decoded = [gopacket.LayerTypeZero]
    df = gopacket.DecodingLayerParser(L.LayerTypeEthernet, ctx=ctx)  # just as a DecodeFeedback
    decoder = dlc.LayersDecoder(L.LayerTypeEthernet, df)
    typ, err = decoder(pktutil.golden_bytes("simple_tcp"), decoded)
    assert err is None and typ == gopacket.LayerTypeZero
    assert len(decoded) == 4
    # the same container behind a parser (decode_test.go:219-232), both panic modes
    for ignore in (True, False):
        p = gopacket.DecodingLayerParser(L.LayerTypeEthernet, ctx=ctx)
        p.SetDecodingLayerContainer(dlc)
        p.IgnorePanic = ignore
        decoded = []
        assert p.DecodeLayers(pktutil.golden_bytes("simple_tcp"), decoded) is None and len(decoded) == 4


def test_layers_decoder_unsupported_and_errors(gp):
    """LayersDecoder's own results (layers_decoder.go:11-101): the first type
    with no decoder comes back without an error (DecodeLayers turns it into
    UnsupportedLayerType), a decoder error with LayerTypeZero, Truncated
    through the feedback, and a first type with no decoder leaves `decoded`
    untouched."""
    gopacket, L, ctx = gp
    dlc = gopacket.DecodingLayerMap().Put(L.Ethernet()).Put(L.IPv4()).Put(L.UDP())
    df = gopacket.DecodingLayerParser(L.LayerTypeEthernet, ctx=ctx)
    dns = pktutil.read_pcap(pktutil.GOLDEN + "/test_dns.pcap")[1][0]
    decoded = []
    typ, err = dlc.LayersDecoder(L.LayerTypeEthernet, df)(dns, decoded)
    assert (typ, err) == (L.LayerTypeDNS, None) and decoded == [L.LayerTypeEthernet, L.LayerTypeIPv4, L.LayerTypeUDP]
    # decode_test.go:1018-1031: a UDP Length past the packet is Truncated, not an error
    full = dlc.Put(L.Dot1Q()).Put(gopacket.Payload())
    decoded, df.Truncated = [], False
    typ, err = full.LayersDecoder(L.LayerTypeEthernet, df)(pktutil.golden_bytes("udp_too_small"), decoded)
    assert (typ, err) == (gopacket.LayerTypeZero, None) and df.Truncated and len(decoded) == 5
    # a decoder error (ip4.go:180-182): LayerTypeZero, the error, the layers before it
    decoded, df.Truncated = [], False
    typ, err = full.LayersDecoder(L.LayerTypeEthernet, df)(pktutil.golden_bytes("simple_tcp")[:20], decoded)
    assert typ == gopacket.LayerTypeZero and err.Error() == "Invalid ip4 header. Length 6 less than 20"
    assert decoded == [L.LayerTypeEthernet] and df.Truncated
    decoded = [L.LayerTypeTCP]
    typ, err = dlc.LayersDecoder(L.LayerTypeTCP, df)(dns, decoded)
    assert (typ, err, decoded) == (L.LayerTypeTCP, None, [L.LayerTypeTCP])


def test_register_port_layer_type_on_device(gp):
    """RegisterTCPPortLayerType (ports.go:99-104) reaches the device parser:
    with port 80 registered as DNS, the simple TCP packet (to port 80) stops
    after TCP with UnsupportedLayerType(DNS), and TCP.NextLayerType() says
    the same; an EthernetTypeMetadata edit (enums.go:310-329) makes an
    unknown EtherType decode as IPv4."""
    gopacket, L, ctx = gp
    L._reset_registry()
    try:
        eth, ip4, tcp = L.Ethernet(), L.IPv4(), L.TCP()
        p = _parser(gp, L.LayerTypeEthernet, eth, ip4, tcp, gopacket.Payload())
        pkt = pktutil.golden_bytes("simple_tcp")
        decoded = []
        assert p.DecodeLayers(pkt, decoded) is None and len(decoded) == 4
        L.RegisterTCPPortLayerType(80, L.LayerTypeDNS)
        err = p.DecodeLayers(pkt, decoded)
        assert err == gopacket.UnsupportedLayerType(L.LayerTypeDNS)
        assert decoded == [L.LayerTypeEthernet, L.LayerTypeIPv4, L.LayerTypeTCP]
        assert tcp.NextLayerType() == L.LayerTypeDNS
        odd = pkt[:12] + b"\x88\xb5" + pkt[14:]
        assert p.DecodeLayers(odd, decoded) is None and decoded == [L.LayerTypeEthernet]  # unknown: success (P1)
        L.EthernetTypeMetadata[0x88B5] = L.EnumMetadata(LayerType=L.LayerTypeIPv4, Name="Local experimental",
                                                        DecodeWith="myDecoder")
        assert p.DecodeLayers(odd, decoded) == gopacket.UnsupportedLayerType(L.LayerTypeDNS)
        assert decoded == [L.LayerTypeEthernet, L.LayerTypeIPv4, L.LayerTypeTCP] and eth.NextLayerType() == 20
        # an entry written without DecodeWith decodes as nothing (enums_generated.go:76-84): LayerTypeZero ends it
        L.EthernetTypeMetadata[0x0800] = L.EnumMetadata(LayerType=L.LayerTypeIPv4, Name="IPv4")
        assert p.DecodeLayers(pkt, decoded) is None and decoded == [L.LayerTypeEthernet]
        assert eth.NextLayerType() == 0
    finally:
        L._reset_registry()


class _Feedback:  # a gopacket.DecodeFeedback that records SetTruncated
    def __init__(self):
        self.truncated = False

    def SetTruncated(self):
        self.truncated = True


def test_decode_from_bytes_one_layer(gp):
    """DecodingLayer.DecodeFromBytes called directly on each struct (the
    interface parser.go:42-60 names): on the device, exactly one header, its
    fields as a full DecodeLayers of the packet sets them."""
    gopacket, L, _ = gp
    pkt = pktutil.golden_bytes("simple_tcp")
    full = [L.Ethernet(), L.IPv4(), L.TCP()]
    assert _parser(gp, L.LayerTypeEthernet, *full, gopacket.Payload()).DecodeLayers(pkt, []) is None
    eth, ip4, tcp = L.Ethernet(), L.IPv4(), L.TCP()
    assert eth.DecodeFromBytes(pkt, gopacket.NilDecodeFeedback) is None
    assert (eth.SrcMAC, eth.DstMAC, eth.EthernetType) == (full[0].SrcMAC, full[0].DstMAC, full[0].EthernetType)
    assert eth.NextLayerType() == L.LayerTypeIPv4 and eth.LayerPayload() == pkt[14:]
    assert ip4.DecodeFromBytes(pkt[14:], gopacket.NilDecodeFeedback) is None
    assert (ip4.SrcIP, ip4.DstIP, ip4.Length, ip4.Checksum) == (full[1].SrcIP, full[1].DstIP, full[1].Length,
                                                                full[1].Checksum)
    assert tcp.DecodeFromBytes(pkt[34:], gopacket.NilDecodeFeedback) is None
    assert (tcp.SrcPort, tcp.DstPort, tcp.Seq, tcp.Window) == (full[2].SrcPort, full[2].DstPort, full[2].Seq,
                                                              full[2].Window)
    assert tcp.LayerPayload() == pkt[66:]


def test_decode_from_bytes_stops_at_its_own_header(gp):
    """A parser of one struct would decode QinQ's inner tag, IP-in-IP's inner
    header, the next IPv6 extension header into the same struct; DecodeFromBytes
    decodes the first one only."""
    gopacket, L, _ = gp
    inner = struct.pack(">HH", (5 << 13) | 300, 0x0800)
    d = L.Dot1Q()
    assert d.DecodeFromBytes(struct.pack(">HH", 100, 0x8100) + inner + bytes(20), gopacket.NilDecodeFeedback) is None
    assert (d.VLANIdentifier, d.Type, d.LayerPayload()[:4]) == (100, 0x8100, inner)
    ipip = bytes.fromhex("4500003c000000004004") + bytes(2) + bytes([10, 0, 0, 1, 10, 0, 0, 2])
    inner4 = bytes.fromhex("45000028000000004006") + bytes(2) + bytes([192, 168, 0, 1, 192, 168, 0, 2])
    ip = L.IPv4()
    assert ip.DecodeFromBytes(ipip + inner4 + bytes(20), gopacket.NilDecodeFeedback) is None
    assert (ip.Protocol, ip.SrcIP, ip.DstIP) == (4, bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2]))
    sk = L.IPv6ExtensionSkipper()
    hbh = bytes([60, 0]) + bytes(6)        # HopByHop, next: Destination options
    dst = bytes([6, 0]) + bytes(6)         # Destination options, next: TCP
    assert sk.DecodeFromBytes(hbh + dst + bytes(20), gopacket.NilDecodeFeedback) is None
    assert sk.NextLayerType() == L.LayerTypeIPv6Destination and sk.LayerPayload() == dst + bytes(20)


def test_decode_from_bytes_errors_and_truncation(gp):
    """Errors come back as the decoder's error value; a truncated header calls
    the DecodeFeedback's SetTruncated (ip4.go:178-271, tcp.go:292-313)."""
    gopacket, L, _ = gp
    from oracle import oracle as O
    pkt = pktutil.golden_bytes("simple_tcp")
    for layer, data, kind in ((L.IPv4(), pkt[14:30], "IPV4"), (L.TCP(), pkt[34:50], "TCP"),
                              (L.IPv4(), bytes([0x42]) + pkt[15:34], "IPV4"), (L.Ethernet(), pkt[:10], "ETHERNET")):
        fb = _Feedback()
        err = layer.DecodeFromBytes(data, fb)
        assert err is not None, (kind, data.hex())
        want = _oracle_error(O, layer, kind, data)
        assert err.Error() == want[0] and fb.truncated == want[1], (kind, err.Error(), want)


def _oracle_error(O, layer, kind, data):
    """The error text and Truncated of a one-decoder parser in the oracle."""
    p = O.OracleParser(int(layer.CanDecode().LayerTypes()[0]), [kind])
    arr = np.frombuffer(data + bytes(16), np.uint8)
    res = p.decode(arr, np.array([0], np.uint64), np.array([len(data)], np.uint32), nthreads=1, layouts=False)
    st = int(res["records"][0]["status"])
    ea = res["err_args"]
    return p.error_string(st & 0x7F, int(ea[0]), int(ea[1])), bool(st & 0x80)


def test_tcp_options_golden(gp):
    """layers/tcp_test.go:88-163 TestPacketTCPOptionDecode / TestPacketMPTCPOptionDecode
    through DecodeLayers: the Options list, the MP_CAPABLE struct included."""
    gopacket, L, _ = gp
    for name, want in (("tcp_option_mss_eol", [L.TCPOption(2, 4, bytes([32, 0])), L.TCPOption(0, 1)]),
                       ("mptcp_capable", [L.TCPOption(2, 4, bytes([32, 0])),
                                          L.TCPOption(30, 4, None, 0, OptionMPTCPMpCapable=L.MPCapable(Version=1)),
                                          L.TCPOption(0, 1)])):
        tcp = L.TCP()
        err = _parser(gp, L.LayerTypeEthernet, L.Ethernet(), L.IPv4(), tcp, gopacket.Payload()).DecodeLayers(
            pktutil.golden_bytes(name), [])
        assert err is None and tcp.Options == want, (name, tcp.Options)
        assert tcp.Padding == b"" or tcp.Padding == bytes(len(tcp.Padding))
