"""The reference API around DecodeLayers in the host mirror (no GPU): the
decoding layer containers (parser.go:48-169), the next-layer registry
(layers/enums.go:294-353, ports.go:54-183: EnumMetadata edits and
Register{TCP,UDP}PortLayerType), the layers' NextLayerType() and CanDecode()
(layerclass.go), checked against the reference's own tables and against the
oracle's decode of the golden packets."""
import pytest

import pktutil
from gopacket_amd import _lib
from gopacket_amd import gopacket as G
from gopacket_amd import layers as L
from oracle import oracle as O


@pytest.fixture(autouse=True)
def clean_registry():
    L._reset_registry()
    yield
    L._reset_registry()


def test_tables_after_init():
    # enums.go:310-353 and the port switches / init() overrides (ports.go, modbus.go:169-171, enip.go:137-140)
    assert L.EthernetTypeLayerType(0x0800) == L.LayerTypeIPv4 and L.EthernetTypeLayerType(0x86DD) == L.LayerTypeIPv6
    assert L.EthernetTypeLayerType(0x8100) == L.LayerTypeDot1Q == L.EthernetTypeLayerType(0x88A8)
    assert L.EthernetTypeLayerType(0x0000) == L.LayerTypeLLC and L.EthernetTypeLayerType(0x1234) == 0
    assert L.IPProtocolLayerType(6) == L.LayerTypeTCP and L.IPProtocolLayerType(0) == L.LayerTypeIPv6HopByHop
    assert L.IPProtocolLayerType(253) == 0 and L.EthernetTypeString(0x1234) == "UnknownEthernetType"
    assert L.TCPPortLayerType(53) == L.LayerTypeDNS and L.TCPPortLayerType(443) == L.LayerTypeTLS
    assert L.TCPPortLayerType(502) == L.LayerTypeModbus  # the init() override beats the switch's ModbusTCP
    assert L.TCPPortLayerType(44818) == L.LayerTypeENIP and L.UDPPortLayerType(2222) == L.LayerTypeENIP
    assert L.TCPPortLayerType(80) == G.LayerTypePayload and L.UDPPortLayerType(53) == L.LayerTypeDNS


def test_registry_edits_reach_parser_config():
    L.RegisterTCPPortLayerType(8080, L.LayerTypeDNS)
    L.EthernetTypeMetadata[0x88B5] = L.EnumMetadata(LayerType=L.LayerTypeIPv4, Name="Local experimental",
                                                    DecodeWith="myDecoder")
    L.IPProtocolMetadata[253] = L.EnumMetadata(LayerType=L.LayerTypeUDP, Name="Experimental", DecodeWith="myDecoder")
    assert L.TCPPortLayerType(8080) == L.LayerTypeDNS and L.EthernetTypeLayerType(0x88B5) == L.LayerTypeIPv4
    assert L.EthernetTypeString(0x88B5) == "Local experimental"
    ed = L._registry_edits()
    assert ed["tcp_port"] == [(8080, int(L.LayerTypeDNS))] and ed["ethertype"] == [(0x88B5, 20)]
    assert ed["ipprotocol"] == [(253, 45)] and ed["udp_port"] == []
    p = G.DecodingLayerParser(L.LayerTypeEthernet, L.Ethernet(), L.IPv4(), L.TCP())
    cfg = p._config()
    assert cfg.decoder_for(L.LayerTypeIPv4) == _lib.DEC_IPV4
    L.RegisterUDPPortLayerType(9999, L.LayerTypeDNS)
    cfg2 = p._config()
    assert cfg2 is not cfg  # an edit rebuilds the device parser
    assert p._config() is cfg2  # ... once
    # Go's in-place form: an unregistered entry has no DecodeWith, so its LayerType()
    # stays 0 and nothing changes (enums_generated.go:146-154); a registered one does
    L.IPProtocolMetadata[254].LayerType = L.LayerTypeTCP
    assert L.IPProtocolLayerType(254) == 0 and L.IPProtocolString(254) == "UnknownIPProtocol"
    assert L._registry_edits()["ipprotocol"] == [(253, 45)] and p._config() is cfg2
    L.IPProtocolMetadata[17].LayerType = L.LayerTypeTCP
    assert L.IPProtocolLayerType(17) == L.LayerTypeTCP and L.IPProtocolString(17) == "UDP"
    assert L._registry_edits()["ipprotocol"] == [(17, 44), (253, 45)] and p._config() is not cfg2


def test_edit_without_decoder_decodes_as_nothing():
    """An EnumMetadata written without DecodeWith: LayerType() 0 and an unknown
    name, as Go's (enums_generated.go:65-84), so the device's table is not changed."""
    L.EthernetTypeMetadata[0x88B5] = L.EnumMetadata(LayerType=L.LayerTypeIPv4, Name="Local experimental")
    assert L.EthernetTypeLayerType(0x88B5) == 0 and L.EthernetTypeString(0x88B5) == "UnknownEthernetType"
    assert L._registry_edits()["ethertype"] == []
    L.EthernetTypeMetadata[0x0800] = L.EnumMetadata(LayerType=L.LayerTypeIPv4, Name="IPv4")  # no decoder now
    assert L.EthernetTypeLayerType(0x0800) == 0 and L._registry_edits()["ethertype"] == [(0x0800, 0)]
    assert L.EthernetTypeMetadata[0x1234].Name == "" and L.EthernetTypeMetadata[0x0800].DecodeWith is None


@pytest.mark.parametrize("form", [G.DecodingLayerMap, G.DecodingLayerSparse, G.DecodingLayerArray])
def test_container_put_and_decoder(form):
    """parser.go:74-169: Put registers every type of CanDecode(), a later Put
    of the same type overrides, Decoder finds it."""
    eth, ip4, skip, skip2 = L.Ethernet(), L.IPv4(), L.IPv6ExtensionSkipper(), L.IPv6ExtensionSkipper()
    dlc = form(None)
    for d in (eth, ip4, skip):
        dlc = dlc.Put(d)
    assert dlc.Decoder(L.LayerTypeEthernet) == (eth, True) and dlc.Decoder(L.LayerTypeIPv4) == (ip4, True)
    for t in L.LayerClassIPv6Extension:
        assert dlc.Decoder(t) == (skip, True)
    assert dlc.Decoder(L.LayerTypeTCP) == (None, False) and dlc.Decoder(5000) == (None, False)
    dlc2 = dlc.Put(skip2)
    assert dlc2.Decoder(L.LayerTypeIPv6Routing) == (skip2, True)
    p = G.DecodingLayerParser(L.LayerTypeEthernet)
    p.SetDecodingLayerContainer(dlc2)
    assert p._decoders == {_lib.DEC_ETHERNET: eth, _lib.DEC_IPV4: ip4, _lib.DEC_IPV6_EXT: skip2}


def test_layer_classes():
    assert L.TCP().CanDecode().Contains(L.LayerTypeTCP) and not L.TCP().CanDecode().Contains(L.LayerTypeUDP)
    assert L.IPv6ExtensionSkipper().CanDecode().LayerTypes() == [46, 47, 48, 49]
    assert G.Payload().CanDecode().LayerTypes() == [G.LayerTypePayload]


def _oracle_structs(first, decoders, pkt):
    """The layer structs of one packet filled from the oracle's layouts (host readers)."""
    names = {L.Ethernet: "ETHERNET", L.Dot1Q: "DOT1Q", L.IPv4: "IPV4", L.IPv6: "IPV6",
             L.IPv6ExtensionSkipper: "IPV6_EXT", L.TCP: "TCP", L.UDP: "UDP", G.Payload: "PAYLOAD"}
    data, off, cap = pktutil.pack([pkt])
    r = O.OracleParser(first, [names[d] for d in decoders]).decode(data, off, cap)
    out = {}
    for slot, kind in enumerate(_lib.LAYOUT_SLOTS):
        s = int(r["layouts"][0]["start"][slot])
        if s == _lib.LAYOUT_ABSENT:
            continue
        for d in decoders:
            if d.kind == kind:
                inst = d()
                inst._hydrate(pkt[s:int(r["layouts"][0]["end"][slot])])
                out[d] = inst
    return out, r


def test_next_layer_type_matches_the_decode():
    """Each struct's NextLayerType() is the type the decode went on to (or
    stopped at): UDP of test_dns.pcap -> DNS (the Unsupported error's type),
    a VLAN-tagged TCP packet's chain Ethernet -> Dot1Q -> IPv4 -> TCP."""
    pkts = pktutil.read_pcap(pktutil.GOLDEN + "/test_dns.pcap")[1]
    decs = (L.Ethernet, L.IPv4, L.UDP)
    for pkt in pkts:
        st, r = _oracle_structs(17, decs, pkt)
        assert int(r["records"][0]["status"]) & _lib.ST_ERR_MASK == 1  # UnsupportedLayerType
        assert st[L.UDP].NextLayerType() == L.LayerTypeDNS == int(r["err_args"][0])
        assert st[L.Ethernet].NextLayerType() == L.LayerTypeIPv4 and st[L.IPv4].NextLayerType() == L.LayerTypeUDP
    decs = (L.Ethernet, L.Dot1Q, L.IPv4, L.TCP, G.Payload)
    st, r = _oracle_structs(17, decs, pktutil.golden_bytes("vlan_tcp"))
    assert (st[L.Ethernet].NextLayerType(), st[L.Dot1Q].NextLayerType(), st[L.IPv4].NextLayerType()) == \
        (L.LayerTypeDot1Q, L.LayerTypeIPv4, L.LayerTypeTCP)


def test_next_layer_type_fragment_and_hopbyhop():
    import struct
    ip = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 40, 7, 0x2000, 64, 6, 0, bytes(4), bytes(4)) + bytes(20)  # MF set
    st, _ = _oracle_structs(20, (L.IPv4,), ip)
    assert st[L.IPv4].NextLayerType() == G.LayerTypeFragment
    st, _ = _oracle_structs(21, (L.IPv6, L.IPv6ExtensionSkipper), pktutil.golden_bytes("ip6_hopbyhop0"))
    assert st[L.IPv6].NextLayerType() == G.LayerTypePayload  # HopByHop.NextHeader 59: NoNextHeader decodes as Payload
