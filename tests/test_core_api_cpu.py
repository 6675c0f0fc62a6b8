"""The root package's helpers around the hot path in the host mirror
(gopacket_amd/gopacket.py): ComputeChecksum / FoldChecksum (checksum.go:35-58),
the LayerType registry (layertype.go:22-111) and the LayerClass forms
(layerclass.go:9-107). Pinned by checksum_test.go:16-50's known answers and
by the device: the mirror's checksum of a packet equals the Correct value of
the engine's decode of it (tests/test_gopacket_api_gpu.py for the device side;
here against the CPU oracle, which the GPU parity tests pin to the device)."""
import struct

import numpy as np
import pytest

import pktutil
from gopacket_amd import gopacket as G
from oracle import oracle as O


@pytest.mark.parametrize("name,want", [("cksum_two_carries", 0xfffe), ("cksum_wikipedia", 0xb861)])
def test_checksum_known_answers(name, want):
    """checksum_test.go:16-50 (the IPv4 header with its checksum field zeroed)."""
    b = bytearray(pktutil.golden_bytes(name))
    b[10] = b[11] = 0
    assert G.FoldChecksum(G.ComputeChecksum(bytes(b))) == want


def test_checksum_against_oracle_and_wrap():
    rng = np.random.default_rng(5)
    for n in (0, 1, 2, 3, 57, 1500, 65537, 262145):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for c0 in (0, 1, 0xFFFF, 0xFFFFFFFF - 3):
            assert G.ComputeChecksum(d, c0) == O.compute_checksum(d, c0)
            assert G.FoldChecksum(G.ComputeChecksum(d, c0)) == O.fold_checksum(O.compute_checksum(d, c0))
    # the sum is a uint32: 70000 words of 0xffff wrap past 2^32 (checksum.go keeps adding)
    assert G.ComputeChecksum(b"\xff\xff" * 70000) == (0xFFFF * 70000) % (1 << 32)
    assert G.FoldChecksum(0) == 0xFFFF and G.FoldChecksum(0xFFFF) == 0 and G.FoldChecksum(0x1FFFE) == 0


def test_layer_type_registry():
    t = G.RegisterLayerType(1777, G.LayerTypeMetadata("Gpk1777"))
    assert t.String() == "Gpk1777" and G.DecodersByLayerName["Gpk1777"] is None
    assert G.UnsupportedLayerType(t).Error() == "No decoder for layer type Gpk1777"
    with pytest.raises(G.GoPanic, match="Layer type already exists"):
        G.RegisterLayerType(1777, G.LayerTypeMetadata("again"))
    with pytest.raises(G.GoPanic, match="Layer type already exists"):
        G.RegisterLayerType(int(G.LayerTypePayload), G.LayerTypeMetadata("Payload2"))
    assert G.OverrideLayerType(1777, G.LayerTypeMetadata("Renamed")).String() == "Renamed"
    assert G.RegisterLayerType(-5, G.LayerTypeMetadata("Negative")).String() == "Negative"  # the map half
    assert G.LayerType(123456).String() == "123456"
    assert G.LayerType(1777).Contains(1777) and G.LayerType(1777).LayerTypes() == [1777]


def test_layer_classes():
    s = G.NewLayerClass([G.LayerType(2), G.LayerType(7)])
    assert isinstance(s, G.LayerClassSlice) and len(s) == 8
    assert s.Contains(7) and not s.Contains(3) and not s.Contains(99) and s.LayerTypes() == [2, 7]
    m = G.NewLayerClass([G.LayerType(2), G.LayerType(2001)])
    assert isinstance(m, G.LayerClassMap) and m.Contains(2001) and not m.Contains(3)
    assert sorted(m.LayerTypes()) == [2, 2001]
    assert isinstance(G.NewLayerClass([G.LayerType(2000)]), G.LayerClassSlice)  # > maxLayerType only


def test_tcp_option_strings_golden():
    """layers/tcp_test.go:17-53 TestTCPOptionKindString."""
    from gopacket_amd import layers as L
    assert L.TCPOption(L.TCPOptionKindNop, 1).String() == "TCPOption(NOP:)"
    assert L.TCPOption(L.TCPOptionKindMSS, 4, b"\x12\x34").String() == "TCPOption(MSS:4660 0x1234)"
    assert L.TCPOption(L.TCPOptionKindTimestamps, 10, bytes([0, 0, 0, 2, 0, 0, 0, 1])).String() == \
        "TCPOption(Timestamps:2/1 0x0000000200000001)"
    assert L.TCPOption(L.TCPOptionKindMultipathTCP, 4, OptionMPTCPMpCapable=L.MPCapable(Version=1)).String() == \
        "MPTCPOption(MP_CAPABLE Version 1)"
    assert L.TCPOption(99, 2, b"").String() == "TCPOption(Unknown(99):)"
    assert L.MPTCPSubtypeString(8) == "MP_TCPRST" and L.MPTCPSubtypeString(12) == "Unknown(12)"


def test_ipv4_flag_option_strings_and_address_to4():
    """ip4.go:28-40, 73-75, 295-321."""
    from gopacket_amd import layers as L
    assert L.IPv4Flag(7).String() == "Evil|DF|MF" and L.IPv4Flag(0).String() == ""
    assert L.IPv4Option(7, 3, b"\x01\x02").String() == "IPv4Option(7:[1 2])"
    assert L.IPv4Option(1, 1).String() == "IPv4Option(1:[])"
    ip = L.IPv4()
    ip.SrcIP, ip.DstIP = bytes(10) + b"\xff\xff\x01\x02\x03\x04", b"\x05\x06\x07\x08"
    assert ip.AddressTo4() is None and (ip.SrcIP, ip.DstIP) == (b"\x01\x02\x03\x04", b"\x05\x06\x07\x08")
    ip.SrcIP = bytes(15) + b"\x01"
    assert ip.AddressTo4().Error() == "Invalid source IPv4 address (address is IPv6)"
    ip.SrcIP, ip.DstIP = b"\x01\x02\x03\x04", b"\x01\x02\x03"
    assert ip.AddressTo4().Error() == "Invalid destination IPv4 address (wrong length of 3 bytes instead of 4)"


def test_mptcp_option_structs():
    """tcp.go:346-527: the option structs built from their bytes, every subtype."""
    from gopacket_amd import layers as L
    opt = lambda L_, st, body: L._mptcp_option(L.TCPOption(30, L_, None, st), bytes([30, L_]) + body)  # noqa
    c = opt(24, 0, bytes([0x01, 0xA5]) + bytes(range(8)) + bytes(range(8, 16)) + b"\x12\x34\x56\x78").OptionMPTCPMpCapable
    assert (c.Version, c.A, c.B, c.C, c.H) == (1, True, False, True, True)
    assert c.SendKey == bytes(range(8)) and c.ReceivKey == bytes(range(8, 16)) and (c.DataLength, c.Checksum) == \
        (0x1234, 0x5678)
    j = opt(12, 1, bytes([0x11, 7]) + struct.pack(">II", 0xAABBCCDD, 99)).OptionMPTCPMpJoin
    assert (j.Backup, j.AddrID, j.ReceivToken, j.SendRandNum, j.SendHMAC) == (True, 7, 0xAABBCCDD, 99, None)
    j = opt(16, 1, bytes([0x10, 3]) + bytes(range(8)) + struct.pack(">I", 5)).OptionMPTCPMpJoin
    assert (j.Backup, j.AddrID, j.SendHMAC, j.SendRandNum) == (False, 3, bytes(range(8)), 5)
    # DSS with an 8-byte data ACK, a 4-byte DSN, SSN, data length and checksum: 4 + 8 + 4 + 4 + 2 + 2 = 24
    d = opt(24, 2, bytes([0x20, 0x07]) + bytes(range(8)) + b"\x00\x00\x00\x09" + struct.pack(">IHH", 77, 1400, 0xBEEF))
    x = d.OptionMPTCPDss
    assert (x.A, x.a, x.M, x.m) == (True, True, True, False) and x.DataAck == bytes(range(8))
    assert (x.DSN, x.SSN, x.DataLength, x.Checksum) == (b"\x00\x00\x00\x09", 77, 1400, 0xBEEF)
    # ADD_ADDR version 1 without the E bit: an HMAC to the end of the options area, an IPv4 address and a port
    a = opt(18, 3, bytes([0x30, 4]) + b"\x0a\x00\x00\x01" + b"\x01\xbb" + bytes(range(8))).OptionMPTCPAddAddr
    assert (a.E, a.AddrID, a.Address, a.Port, a.SendHMAC) == (False, 4, b"\x0a\x00\x00\x01", 443, bytes(range(8)))
    assert opt(6, 4, bytes([0x40, 1, 2, 3])).OptionMTCPRemAddr.AddrIDs == [1, 2, 3]
    p = opt(4, 5, bytes([0x51, 9])).OptionMPTCPMpPrio
    assert (p.Backup, p.AddrID) == (True, 9)
    assert opt(12, 6, bytes([0x60, 0]) + struct.pack(">Q", 2 ** 40)).OptionMTCPMPFail.DSN == 2 ** 40
    assert opt(12, 7, bytes([0x70, 0]) + bytes(range(8))).OptionMTCPMPFastClose.ReceivKey == bytes(range(8))
    r = opt(4, 8, bytes([0x8B, 5])).OptionMPTCPMPTcpRst
    assert (r.U, r.V, r.W, r.T, r.Reason) == (True, False, True, True, 5)
    assert str(L.TCPOption(30, 4, None, 8, OptionMPTCPMPTcpRst=r)) == "MPTCPOption(MP_TCPRST Transient true; Reason 5)"


def test_tcp_compute_checksum_and_network_layer():
    """tcp.go:251-257 ComputeChecksum over tcpip.go:19-85's pseudo-header:
    0 over a correct segment, the checksum itself with the field zeroed
    (simple_tcp's 0x9a8f, decode_test.go:386-492); the errors without a
    network layer or with a non-IP one; IPv6.AddressTo16 (ip6.go:742-761)."""
    from gopacket_amd import layers as L
    pkt = pktutil.golden_bytes("simple_tcp")
    ip4, tcp = L.IPv4(), L.TCP()
    ip4._hydrate(pkt[14:])
    tcp._hydrate(pkt[34:34 + ip4.Length - 20])
    csum, err = tcp.ComputeChecksum()
    assert csum == 0 and err.Error().startswith("TCP/IP layer 4 checksum cannot be computed without network layer")
    assert tcp.SetNetworkLayerForChecksum(L.Ethernet()).Error() == \
        "cannot use layer type Ethernet for tcp checksum network layer"
    assert tcp.SetNetworkLayerForChecksum(ip4) is None
    assert tcp.ComputeChecksum() == (0, None)
    tcp.Contents = tcp.Contents[:16] + b"\x00\x00" + tcp.Contents[18:]
    assert tcp.ComputeChecksum() == (0x9a8f, None)
    ip6 = L.IPv6()
    ip6.SrcIP, ip6.DstIP = bytes(16), b"\x01\x02\x03\x04"
    assert ip6.AddressTo16().Error() == "Invalid destination IPv6 address (address is IPv4)"
    assert tcp.SetNetworkLayerForChecksum(ip6) is None
    assert tcp.ComputeChecksum()[1].Error() == "Invalid destination IPv6 address (address is IPv4)"
    ip6.DstIP = bytes(15) + b"\x01"
    assert ip6.AddressTo16() is None and tcp.ComputeChecksum()[1] is None
