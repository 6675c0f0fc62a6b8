"""The Endpoint / Flow interface of the host mirror (gopacket_amd/gopacket.py,
layers.py; flows.go:27-236, layers/endpoints.go:17-99): constructors, the
registry of endpoint types and their String forms, LessThan, FlowFromEndpoints,
and FastHash of hand-built flows against the same flows the device hashed.
Pinned by layers/endpoints_test.go:16-37 (TestNewIPEndpoint) and by Go's
formatting rules (net.IP / net.HardwareAddr String, fmt's %v of a byte array)."""
import ipaddress

import pytest

from gopacket_amd import gopacket as G
from gopacket_amd import layers as L


def test_new_ip_endpoint_golden():
    """layers/endpoints_test.go:16-37: To4 and To16 forms of 192.168.0.1 give IPv4, a v6 address IPv6."""
    v4 = ipaddress.ip_address("192.168.0.1").packed
    mapped = bytes(10) + b"\xff\xff" + v4  # net.ParseIP(...).To16()
    v6 = ipaddress.ip_address("2001:0db8:85a3:0000:0000:8a2e:0370:7334").packed
    for ip, typ in ((v4, G.EndpointIPv4), (mapped, G.EndpointIPv4), (v6, G.EndpointIPv6)):
        e = L.NewIPEndpoint(ip)
        assert e != G.InvalidEndpoint and e.EndpointType() == typ
    assert L.NewIPEndpoint(b"\x01\x02\x03") == G.InvalidEndpoint
    assert L.NewIPEndpoint(mapped).Raw() == v4


def test_endpoint_strings():
    assert str(L.NewIPEndpoint(ipaddress.ip_address("10.0.0.1"))) == "10.0.0.1"
    assert str(L.NewIPEndpoint(ipaddress.ip_address("2001:db8::8a2e:370:7334"))) == "2001:db8::8a2e:370:7334"
    assert str(G.NewEndpoint(G.EndpointIPv6, bytes(10) + b"\xff\xff\x01\x02\x03\x04")) == "1.2.3.4"  # net.IP.String
    assert str(L.NewMACEndpoint(b"\x00\x1b\x21\x0a\x0b\x0c")) == "00:1b:21:0a:0b:0c"
    assert str(L.NewTCPPortEndpoint(443)) == "443" and str(L.NewUDPPortEndpoint(53)) == "53"
    assert str(L.NewSCTPPortEndpoint(9)) == "9" and str(L.NewUDPLitePortEndpoint(7)) == "7"
    assert str(L.NewRUDPPortEndpoint(300)) == "44"  # byte(p)
    assert str(G.NewEndpoint(G.EndpointPPP, b"")) == "point"
    assert str(G.InvalidEndpoint) == "[]" and str(G.InvalidFlow) == "[]->[]"
    # an unregistered type: "%v:%v" of the type number and the whole [16]byte array
    assert str(G.NewEndpoint(4242, b"\x01\x02")) == "4242:[1 2" + " 0" * 14 + "]"
    assert G.EndpointType(4242).String() == "4242" and G.EndpointTCPPort.String() == "TCP"
    f = G.NewFlow(G.EndpointTCPPort, b"\x00\x50", b"\x1f\x90")
    assert str(f) == "80->8080" and str(f.Reverse()) == "8080->80"


def test_register_endpoint_type():
    t = G.RegisterEndpointType(31337, G.EndpointTypeMetadata("Mine", lambda b: "mine:" + b.hex()))
    assert t.String() == "Mine" and str(G.NewEndpoint(t, b"\xab")) == "mine:ab"
    with pytest.raises(G.GoPanic, match="Endpoint type number already in use"):
        G.RegisterEndpointType(31337, G.EndpointTypeMetadata("Again"))
    with pytest.raises(G.GoPanic, match="Endpoint type number already in use"):
        G.RegisterEndpointType(4, G.EndpointTypeMetadata("TCP again"))


def test_less_than_and_size_limits():
    a, b = L.NewIPEndpoint(b"\x0a\x00\x00\x01"), L.NewIPEndpoint(b"\x0a\x00\x00\x02")
    six = L.NewIPEndpoint(bytes(15) + b"\x01")
    assert a.LessThan(b) and not b.LessThan(a) and not a.LessThan(a)
    assert a.LessThan(six) and b.LessThan(six)  # IPv6 > IPv4 for all addresses (endpoints.go:18-20)
    assert G.NewEndpoint(1, b"\x01").LessThan(G.NewEndpoint(1, b"\x01\x00"))  # bytes.Compare: shorter first
    with pytest.raises(G.GoPanic, match="raw byte length greater than MaxEndpointSize"):
        G.NewEndpoint(1, bytes(17))
    with pytest.raises(G.GoPanic, match="flow raw byte length greater than MaxEndpointSize"):
        G.NewFlow(1, bytes(17), b"")


def test_flow_from_endpoints():
    s, d = L.NewTCPPortEndpoint(1000), L.NewTCPPortEndpoint(80)
    f, err = G.FlowFromEndpoints(s, d)
    assert err is None and f == G.NewFlow(G.EndpointTCPPort, s.Raw(), d.Raw())
    assert f.Endpoints() == (s, d) and f.Src() == s and f.Dst() == d
    assert f.FastHash() == f.Reverse().FastHash() == G.NewFlow(G.EndpointTCPPort, d.Raw(), s.Raw()).FastHash()
    _, err = G.FlowFromEndpoints(s, L.NewUDPPortEndpoint(80))
    assert err.Error() == "Mismatched endpoint types: TCP->UDP"
    # FNV-1a of the raw bytes, the type folded in (flows.go:78-83, 167-174)
    e = L.NewIPEndpoint(b"\x01\x02\x03\x04")
    h = 14695981039346656037
    for x in b"\x01\x02\x03\x04":
        h = ((h ^ x) * 1099511628211) & (2 ** 64 - 1)
    assert e.FastHash() == ((h ^ 1) * 1099511628211) & (2 ** 64 - 1)
