"""gopacket/layers surface for the hot path: LayerType and enum constants and
the DecodingLayer structs Ethernet, Dot1Q, IPv4, IPv6, IPv6ExtensionSkipper,
TCP, UDP (layers/{ethernet,dot1q,ip4,ip6,tcp,udp}.go).

These structs are filled from device results, in one of two ways:
- _fill(pkt, s, e, f): from the gpk_fields record the device wrote for the
  packet (gpk_decode_batch_fields) and the slice [s, e) its DecodeFromBytes
  was handed (derived from the decoded list, gopacket.BatchResult.Hydrate):
  every scalar field is the record's, option lists come from the record's
  option start maps, and Contents/Payload are slices at the header length and
  payload end the record's fields give. No header is decoded on the host.
- _hydrate(d): from the slice alone (a gpk_layout range), every field a pure
  read of those packet bytes, following the field assignments of the
  reference decoder it names; the fallback for what the record does not hold.
Option lists are walked from bytes whose validity the device already
established (the device reports any option error as the packet's error).
"""
import json
import os
import struct
from dataclasses import dataclass, field
from typing import List, Optional

from . import _lib
from .gopacket import (ChecksumVerificationResult, Flow, LayerClass, LayerType, NewFlow, EndpointIPv4, EndpointIPv6,
                       EndpointMAC, EndpointTCPPort, EndpointUDPPort, EndpointSCTPPort, EndpointRUDPPort,
                       EndpointUDPLitePort, EndpointPPP, InvalidEndpoint, NewEndpoint, LayerTypeFragment,
                       LayerTypePayload)

_REG = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "registry_gen.json")))

# ---- LayerType constants (layers/layertypes.go) -----------------------------
_by_name = {}
for _id, _name in _REG["layer_type_names"].items():
    _by_name.setdefault(_name, int(_id))


def _lt(name):
    return LayerType(_by_name[name])


LayerTypeARP = _lt("ARP")
LayerTypeDot1Q = _lt("Dot1Q")
LayerTypeEthernet = _lt("Ethernet")
LayerTypeICMPv4 = _lt("ICMPv4")
LayerTypeIPv4 = _lt("IPv4")
LayerTypeIPv6 = _lt("IPv6")
LayerTypeLLC = _lt("LLC")
LayerTypeTCP = _lt("TCP")
LayerTypeUDP = _lt("UDP")
LayerTypeIPv6HopByHop = _lt("IPv6HopByHop")
LayerTypeIPv6Routing = _lt("IPv6Routing")
LayerTypeIPv6Fragment = _lt("IPv6Fragment")
LayerTypeIPv6Destination = _lt("IPv6Destination")
LayerTypeDNS = _lt("DNS")
LayerTypeTLS = _lt("TLS")
LayerTypeModbus = _lt("Modbus")
LayerTypeENIP = _lt("ENIP")
# layertypes.go:200-206
LayerClassIPv6Extension = LayerClass([LayerTypeIPv6HopByHop, LayerTypeIPv6Routing, LayerTypeIPv6Fragment,
                                      LayerTypeIPv6Destination])

# ---- enums (layers/enums.go) -------------------------------------------------
EthernetTypeLLC = 0x0000
EthernetTypeIPv4 = 0x0800
EthernetTypeARP = 0x0806
EthernetTypeIPv6 = 0x86DD
EthernetTypeDot1Q = 0x8100
EthernetTypeQinQ = 0x88A8
IPProtocolIPv6HopByHop = 0
IPProtocolTCP = 6
IPProtocolUDP = 17
IPProtocolIPv4 = 4
IPProtocolIPv6 = 41
IPProtocolNoNextHeader = 59
IPv6HopByHopOptionJumbogram = 0xC2

_IPPROTO_NAMES = {v: n for v, lt, n in _REG["ipprotocol"]}
_ETHERTYPE_NAMES = {v: n for v, lt, n in _REG["ethertype"]}


def IPProtocolString(p):
    """IPProtocol.String() (enums_generated.go:135-143)"""
    return IPProtocolMetadata._name(int(p))


def EthernetTypeString(t):
    """EthernetType.String() (enums_generated.go:65-73)"""
    return EthernetTypeMetadata._name(int(t))


# ---- next-layer tables (layers/enums.go:294-390, ports.go:54-183) -----------
# The registry the reference's NextLayerType methods consult, as the host
# mirror: EthernetTypeMetadata / IPProtocolMetadata (EnumMetadata per value,
# enums.go:294-353, editable as in Go) and the TCP/UDP port overrides of
# RegisterTCPPortLayerType / RegisterUDPPortLayerType (ports.go:95-104,
# 174-183) over the port switches. Every DecodingLayerParser built after an
# edit sends the edited entries to its device parser (gpk_parser_set_*), so
# the device's NextLayerType lookups and the structs' NextLayerType() agree.


class EnumMetadata:
    """enums.go EnumMetadata: the decoder, the name and the LayerType of a
    value. Go's EthernetType / IPProtocol LayerType() and String() read an
    entry only when its DecodeWith is set (enums_generated.go:65-84,
    135-154): an entry written without one decodes as nothing (LayerType 0)
    and prints as unknown, whatever its LayerType and Name say."""

    def __init__(self, LayerType=0, Name="", DecodeWith=None):
        self.LayerType, self.Name, self.DecodeWith = LayerType, Name, DecodeWith

    def __repr__(self):
        return "EnumMetadata(LayerType=%d, Name=%r, DecodeWith=%r)" % (int(self.LayerType), self.Name,
                                                                       self.DecodeWith)


class _GoDecoder:
    """The DecodeWith of an entry initActualTypeData registered (enums.go:310-353):
    a decoder of the reference's NewPacket path, which the hot path never calls."""

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return "decode%s" % self.name


class _EnumTable:
    """A [n]EnumMetadata array: the generated defaults, and every entry a
    caller has touched kept as its own object, so both forms of Go's edit
    work: `T[v] = EnumMetadata(...)` and `T[v].LayerType = ...`."""

    def __init__(self, rows, n, unknown):
        self._default = {v: (LayerType(lt), name) for v, lt, name in rows}
        self._n, self._unknown, self._edits = n, unknown, {}

    def _effective(self, v):
        """What Go's LayerType() returns for v (0 without a DecodeWith)."""
        m = self._edits.get(v)
        if m is None:
            return int(self._default.get(v, (0, ""))[0])
        return int(m.LayerType) if m.DecodeWith is not None else 0

    def _name(self, v):
        m = self[v]
        return m.Name if m.DecodeWith is not None else self._unknown

    def _check(self, v):
        v = int(v)
        if not 0 <= v < self._n:
            raise IndexError(v)
        return v

    def __getitem__(self, v):
        v = self._check(v)
        if v not in self._edits:
            if v in self._default:
                lt, name = self._default[v]
                self._edits[v] = EnumMetadata(lt, name, _GoDecoder(name))
            else:  # the zero EnumMetadata: no decoder
                self._edits[v] = EnumMetadata(LayerType(0), "", None)
        return self._edits[v]

    def __setitem__(self, v, meta):
        self._edits[self._check(v)] = meta

    def _changed(self):
        """(value, LayerType) of every entry whose effective LayerType differs from the default."""
        out = []
        for v in sorted(self._edits):
            lt = self._effective(v)
            if lt != int(self._default.get(v, (0, ""))[0]):
                out.append((v, lt))
        return out


EthernetTypeMetadata = _EnumTable(_REG["ethertype"], 65536, "UnknownEthernetType")
IPProtocolMetadata = _EnumTable(_REG["ipprotocol"], 256, "UnknownIPProtocol")

_TCP_SWITCH = {p: LayerType(lt) for p, lt in _REG["tcp_port_switch"]}
_UDP_SWITCH = {p: LayerType(lt) for p, lt in _REG["udp_port_switch"]}
_tcp_override = {p: LayerType(lt) for p, lt in _REG["tcp_port_override"]}  # init() registrations
_udp_override = {p: LayerType(lt) for p, lt in _REG["udp_port_override"]}
_tcp_user, _udp_user = {}, {}


def RegisterTCPPortLayerType(port, layerType):
    """ports.go:99-104"""
    _tcp_override[int(port)] = _tcp_user[int(port)] = LayerType(layerType)


def RegisterUDPPortLayerType(port, layerType):
    """ports.go:178-183"""
    _udp_override[int(port)] = _udp_user[int(port)] = LayerType(layerType)


def EthernetTypeLayerType(t):
    """EthernetType.LayerType() (enums_generated.go:76-84)."""
    return LayerType(EthernetTypeMetadata._effective(EthernetTypeMetadata._check(t)))


def IPProtocolLayerType(p):
    """IPProtocol.LayerType() (enums_generated.go:146-154)."""
    return LayerType(IPProtocolMetadata._effective(IPProtocolMetadata._check(p)))


def TCPPortLayerType(port):
    """TCPPort.LayerType() (ports.go:54-93): the override, else the switch, else Payload."""
    port = int(port)
    if port in _tcp_override:
        return _tcp_override[port]
    return _TCP_SWITCH.get(port, LayerTypePayload)


def UDPPortLayerType(port):
    """UDPPort.LayerType() (ports.go:121-172)."""
    port = int(port)
    if port in _udp_override:
        return _udp_override[port]
    return _UDP_SWITCH.get(port, LayerTypePayload)


def _reset_registry():
    """Back to the reference's registry after init() (tests)."""
    EthernetTypeMetadata._edits.clear()
    IPProtocolMetadata._edits.clear()
    _tcp_user.clear()
    _udp_user.clear()
    _tcp_override.clear()
    _tcp_override.update({p: LayerType(lt) for p, lt in _REG["tcp_port_override"]})
    _udp_override.clear()
    _udp_override.update({p: LayerType(lt) for p, lt in _REG["udp_port_override"]})


def _registry_edits():
    """What a device parser must be told beyond its default tables."""
    return dict(ethertype=EthernetTypeMetadata._changed(), ipprotocol=IPProtocolMetadata._changed(),
                tcp_port=sorted((p, int(lt)) for p, lt in _tcp_user.items()),
                udp_port=sorted((p, int(lt)) for p, lt in _udp_user.items()))


def _be16(b, o):
    return (b[o] << 8) | b[o + 1]


def _be32(b, o):
    return struct.unpack_from(">I", b, o)[0]


_NO_DECODER = 1999  # a LayerType no device parser has a decoder for


def _tables_into(own):
    """(value, LayerType) entries that send every next-layer lookup landing on
    one of the types in `own` to a type without a decoder instead."""
    def enum(t):
        vals = set(t._default) | set(t._edits)
        return [(v, _NO_DECODER) for v in sorted(vals) if t._effective(v) in own]

    def ports(switch, override, lookup):
        return [(p, _NO_DECODER) for p in sorted(set(switch) | set(override)) if int(lookup(p)) in own]

    return dict(ethertype=enum(EthernetTypeMetadata), ipprotocol=enum(IPProtocolMetadata),
                tcp_port=ports(_TCP_SWITCH, _tcp_override, TCPPortLayerType),
                udp_port=ports(_UDP_SWITCH, _udp_override, UDPPortLayerType))


class BaseLayer:
    Contents: bytes = b""
    Payload: bytes = b""

    def LayerContents(self):
        return self.Contents

    def LayerPayload(self):
        return self.Payload

    def DecodeFromBytes(self, data, df):
        """The DecodingLayer method (ethernet.go:42-63, dot1q.go:30-41,
        ip4.go:178-271, ip6.go:221-278, 443-451, tcp.go:291-551, udp.go:30-56),
        on the device: one packet through a parser holding only this layer,
        whose next-layer tables lead nowhere back into it, so exactly this one
        header is decoded. Returns the decoder's error (None on success); a
        truncated header calls df.SetTruncated(); a decoder panic raises
        GoPanic, as it propagates out of DecodeFromBytes in Go."""
        from .gopacket import DecodingLayerArray, _LayersDecoder
        types = self.CanDecode().LayerTypes()
        dec = _LayersDecoder(DecodingLayerArray().Put(self), types[0], df, _tables_into({int(t) for t in types}))
        _, err = dec(bytes(data), [])
        return err


# ---- layers/ethernet.go:22-63 ------------------------------------------------
class Ethernet(BaseLayer):
    kind = _lib.DEC_ETHERNET

    def __init__(self):
        self.SrcMAC = self.DstMAC = b""
        self.EthernetType = 0
        self.Length = 0

    def LayerType(self):
        return LayerTypeEthernet

    def CanDecode(self):
        return LayerClass([LayerTypeEthernet])

    def _hydrate(self, d):
        self.DstMAC = d[0:6]
        self.SrcMAC = d[6:12]
        self.EthernetType = _be16(d, 12)
        self.Contents, self.Payload = d[:14], d[14:]
        self._poff = 14
        self.Length = 0
        if self.EthernetType < 0x0600:
            self.Length = self.EthernetType
            self.EthernetType = EthernetTypeLLC
            if len(self.Payload) > self.Length:
                self.Payload = self.Payload[:self.Length]

    def _fill(self, pkt, s, e, f):
        self.DstMAC, self.SrcMAC = bytes(f["eth_dst"]), bytes(f["eth_src"])
        self.EthernetType, self.Length = int(f["eth_type"]), int(f["eth_length"])
        self.Contents, self.Payload = pkt[s:s + 14], pkt[s + 14:payload_end(_lib.DEC_ETHERNET, pkt, s, e, f)]
        self._poff = 14

    def NextLayerType(self):
        """ethernet.go:111-113"""
        return EthernetTypeLayerType(self.EthernetType)

    def LinkFlow(self):
        return NewFlow(EndpointMAC, self.SrcMAC, self.DstMAC)


# ---- layers/dot1q.go:17-41 ---------------------------------------------------
class Dot1Q(BaseLayer):
    kind = _lib.DEC_DOT1Q

    def __init__(self):
        self.Priority = 0
        self.DropEligible = False
        self.VLANIdentifier = 0
        self.Type = 0

    def LayerType(self):
        return LayerTypeDot1Q

    def CanDecode(self):
        return LayerClass([LayerTypeDot1Q])

    def _hydrate(self, d):
        self.Priority = (d[0] & 0xE0) >> 5
        self.DropEligible = d[0] & 0x10 != 0
        self.VLANIdentifier = _be16(d, 0) & 0x0FFF
        self.Type = _be16(d, 2)
        self.Contents, self.Payload = d[:4], d[4:]
        self._poff = 4

    def _fill(self, pkt, s, e, f):
        tci = int(f["d1q_tci"])
        self.Priority, self.DropEligible, self.VLANIdentifier = tci >> 13, bool(tci >> 12 & 1), tci & 0x0FFF
        self.Type = int(f["d1q_type"])
        self.Contents, self.Payload = pkt[s:s + 4], pkt[s + 4:e]
        self._poff = 4

    def NextLayerType(self):
        """dot1q.go:49-51"""
        return EthernetTypeLayerType(self.Type)


IPv4EvilBit, IPv4DontFragment, IPv4MoreFragments = 1 << 2, 1 << 1, 1 << 0


class IPv4Flag(int):
    """ip4.go:22-40"""

    def String(self):
        names = [n for bit, n in ((IPv4EvilBit, "Evil"), (IPv4DontFragment, "DF"), (IPv4MoreFragments, "MF"))
                 if self & bit]
        return "|".join(names)

    __str__ = String


@dataclass
class IPv4Option:
    OptionType: int = 0
    OptionLength: int = 0
    OptionData: Optional[bytes] = None

    def String(self):  # ip4.go:73-75: "IPv4Option(%v:%v)"
        return "IPv4Option(%d:[%s])" % (self.OptionType, " ".join(str(b) for b in (self.OptionData or b"")))

    __str__ = String


class _Checksummed:
    _csum = None  # (error, ChecksumVerificationResult) set from the device record
    _pseudoheader = None  # tcpipchecksum.pseudoheader (TCP, UDP)

    def SetNetworkLayerForChecksum(self, l):
        """tcpip.go:75-85 (TCP and UDP): the IPv4 or IPv6 layer whose addresses
        the pseudo-header of ComputeChecksum uses."""
        from .gopacket import GoError
        if not hasattr(l, "_pseudoheader_checksum"):
            return GoError("cannot use layer type %s for tcp checksum network layer" % l.LayerType().String())
        self._pseudoheader = l
        return None

    def _compute_checksum(self, header_and_payload, proto):
        """tcpipchecksum.computeChecksum (tcpip.go:44-62): (uint32 sum, error)."""
        from .gopacket import ComputeChecksum, GoError
        if self._pseudoheader is None:
            return 0, GoError("TCP/IP layer 4 checksum cannot be computed without network layer... "
                              "call SetNetworkLayerForChecksum to set which layer to use")
        n = len(header_and_payload)
        csum, err = self._pseudoheader._pseudoheader_checksum()
        if err is not None:
            return 0, err
        csum += proto + (n & 0xFFFF) + (n >> 16)
        return ComputeChecksum(header_and_payload, csum & 0xFFFFFFFF), None

    def VerifyChecksum(self):
        """The device's checksum verification of this layer (see DecodingLayerParser)."""
        if self._csum is None:
            raise RuntimeError("no device checksum result attached to this layer")
        return self._csum


# ---- layers/ip4.go:42-271 ----------------------------------------------------
class IPv4(BaseLayer, _Checksummed):
    kind = _lib.DEC_IPV4

    def __init__(self):
        self.Version = self.IHL = self.TOS = 0
        self.Length = self.Id = 0
        self.Flags = self.FragOffset = 0
        self.TTL = self.Protocol = self.Checksum = 0
        self.SrcIP = self.DstIP = b""
        self.Options: List[IPv4Option] = []
        self.Padding = None

    def LayerType(self):
        return LayerTypeIPv4

    def CanDecode(self):
        return LayerClass([LayerTypeIPv4])

    def _hydrate(self, d):
        self.Length = _be16(d, 2)
        self.IHL = d[0] & 0x0F
        if self.Length == 0:
            self.Length = len(d) & 0xFFFF
        if len(d) > self.Length:
            d = d[:self.Length]
        hl = self.IHL * 4
        self.Options = []
        self.Contents, self.Payload = d[:hl], d[hl:]
        opts = d[20:hl]
        while len(opts) > 0:
            t = opts[0]
            if t == 0:
                self.Options.append(IPv4Option(0, 1))
                self.Padding = opts[1:]
                break
            if t == 1:
                self.Options.append(IPv4Option(1, 1))
                opts = opts[1:]
                continue
            ol = opts[1]
            self.Options.append(IPv4Option(t, ol, opts[2:ol]))
            opts = opts[ol:]
        ff = _be16(d, 6)
        self.Version = d[0] >> 4
        self.TOS = d[1]
        self.Id = _be16(d, 4)
        self.Flags = IPv4Flag(ff >> 13)
        self.FragOffset = ff & 0x1FFF
        self.TTL = d[8]
        self.Protocol = d[9]
        self.Checksum = _be16(d, 10)
        self.SrcIP = d[12:16]
        self.DstIP = d[16:20]
        self._poff = hl

    def _fill(self, pkt, s, e, f):
        self.Version, self.IHL, self.TOS = int(f["ip4_version"]), int(f["ip4_ihl"]), int(f["ip4_tos"])
        self.Length, self.Id = int(f["ip4_length"]), int(f["ip4_id"])
        ff = int(f["ip4_flags_frag"])
        self.Flags, self.FragOffset = IPv4Flag(ff >> 13), ff & 0x1FFF
        self.TTL, self.Protocol, self.Checksum = int(f["ip4_ttl"]), int(f["ip4_protocol"]), int(f["ip4_checksum"])
        self.SrcIP, self.DstIP = bytes(f["ip4_src"]), bytes(f["ip4_dst"])
        hl = self.IHL * 4
        self.Contents, self.Payload = pkt[s:s + hl], pkt[s + hl:payload_end(_lib.DEC_IPV4, pkt, s, e, f)]
        self.Options, padding = IPv4OptionsFromMap(pkt, s, hl, f["ip4_opt_map"])
        if padding is not None:  # set only by an End of options (ip4.go:231), else kept
            self.Padding = padding
        self._poff = hl

    def NextLayerType(self):
        """ip4.go:277-282: a fragment (MoreFragments or an offset) decodes as Fragment"""
        if self.Flags & 1 or self.FragOffset != 0:
            return LayerTypeFragment
        return IPProtocolLayerType(self.Protocol)

    def NetworkFlow(self):
        return NewFlow(EndpointIPv4, self.SrcIP, self.DstIP)

    def AddressTo4(self):
        """ip4.go:295-321: both addresses in their 4-byte form, or the error."""
        from .gopacket import GoError

        def check(a):
            c = _to4(bytes(a))
            if c is not None:
                return c, None
            if len(a) == 16:
                return None, "address is IPv6"
            return None, "wrong length of %d bytes instead of 4" % len(a)

        src, e = check(self.SrcIP)
        if e:
            return GoError("Invalid source IPv4 address (%s)" % e)
        dst, e = check(self.DstIP)
        if e:
            return GoError("Invalid destination IPv4 address (%s)" % e)
        self.SrcIP, self.DstIP = src, dst
        return None

    def _pseudoheader_checksum(self):  # tcpip.go:19-28
        err = self.AddressTo4()
        if err is not None:
            return 0, err
        s_, d_ = self.SrcIP, self.DstIP
        csum = ((s_[0] + s_[2]) << 8) + s_[1] + s_[3] + ((d_[0] + d_[2]) << 8) + d_[1] + d_[3]
        return csum, None


@dataclass
class IPv6HopByHopOption:
    OptionType: int = 0
    OptionLength: int = 0
    ActualLength: int = 0
    OptionData: Optional[bytes] = None


class IPv6HopByHop(BaseLayer):
    def __init__(self):
        self.NextHeader = 0
        self.HeaderLength = 0
        self.ActualLength = 0
        self.Options: List[IPv6HopByHopOption] = []

    def LayerType(self):
        return LayerTypeIPv6HopByHop


# ---- layers/ip6.go:28-278 ----------------------------------------------------
class IPv6(BaseLayer, _Checksummed):
    kind = _lib.DEC_IPV6

    def __init__(self):
        self.Version = self.TrafficClass = self.FlowLabel = 0
        self.Length = self.NextHeader = self.HopLimit = 0
        self.SrcIP = self.DstIP = b""
        self.HopByHop = None
        self.hbh = IPv6HopByHop()

    def LayerType(self):
        return LayerTypeIPv6

    def CanDecode(self):
        return LayerClass([LayerTypeIPv6])

    def _hydrate(self, d):
        self.Version = d[0] >> 4
        self.TrafficClass = (_be16(d, 0) >> 4) & 0xFF
        self.FlowLabel = _be32(d, 0) & 0x000FFFFF
        self.Length = _be16(d, 4)
        self.NextHeader = d[6]
        self.HopLimit = d[7]
        self.SrcIP, self.DstIP = d[8:24], d[24:40]
        self.HopByHop = None
        self.Contents, self.Payload = d[:40], d[40:]
        if self.NextHeader == IPProtocolIPv6HopByHop:
            h, p = self.hbh, self.Payload
            h.NextHeader, h.HeaderLength = p[0], p[1]
            h.ActualLength = p[1] * 8 + 8
            h.Contents, h.Payload = p[:h.ActualLength], p[h.ActualLength:]
            h.Options = []
            off = 2
            while off < h.ActualLength:
                if p[off] == 0:
                    o = IPv6HopByHopOption(0, 0, 1, None)
                else:
                    al = p[off + 1] + 2
                    o = IPv6HopByHopOption(p[off], p[off + 1], al, p[off + 2:off + al])
                h.Options.append(o)
                off += o.ActualLength
            self.HopByHop = h
            jumbo = next((o for o in h.Options if o.OptionType == IPv6HopByHopOptionJumbogram), None)
            if jumbo is not None and self.Length == 0:
                self.Payload = self.Payload[:min(_be32(jumbo.OptionData, 0), len(self.Payload))]
                self._poff = 40
                return
            self.Payload = self.Payload[h.ActualLength:]
        self.Payload = self.Payload[:min(self.Length, len(self.Payload))]
        self._poff = 40 + (self.hbh.ActualLength if self.HopByHop is not None else 0)

    def _fill(self, pkt, s, e, f):
        self.Version, self.TrafficClass = int(f["ip6_version"]), int(f["ip6_traffic_class"])
        self.FlowLabel, self.Length = int(f["ip6_flow_label"]), int(f["ip6_length"])
        self.NextHeader, self.HopLimit = int(f["ip6_next_header"]), int(f["ip6_hop_limit"])
        self.SrcIP, self.DstIP = bytes(f["ip6_src"]), bytes(f["ip6_dst"])
        self.HopByHop = None
        self.Contents = pkt[s:s + 40]
        if self.NextHeader == IPProtocolIPv6HopByHop:
            HopByHopFromMap(self.hbh, pkt, s + 40, e, f["hbh_opt_map"])
            self.HopByHop = self.hbh
        self._poff = ipv6_payload_start(pkt, s, f) - s
        self.Payload = pkt[s + self._poff:payload_end(_lib.DEC_IPV6, pkt, s, e, f)]

    def NextLayerType(self):
        """ip6.go:286-291"""
        if self.HopByHop is not None:
            return IPProtocolLayerType(self.HopByHop.NextHeader)
        return IPProtocolLayerType(self.NextHeader)

    def NetworkFlow(self):
        return NewFlow(EndpointIPv6, self.SrcIP, self.DstIP)

    def AddressTo16(self):
        """ip6.go:742-761: an error unless both addresses are 16 bytes."""
        from .gopacket import GoError
        for which, a in (("source", self.SrcIP), ("destination", self.DstIP)):
            if len(a) != 16:
                e = "address is IPv4" if len(a) == 4 else "wrong length of %d bytes instead of 16" % len(a)
                return GoError("Invalid %s IPv6 address (%s)" % (which, e))
        return None

    def _pseudoheader_checksum(self):  # tcpip.go:30-42
        err = self.AddressTo16()
        if err is not None:
            return 0, err
        csum = 0
        for i in range(0, 16, 2):
            csum += (self.SrcIP[i] << 8) + self.SrcIP[i + 1] + (self.DstIP[i] << 8) + self.DstIP[i + 1]
        return csum & 0xFFFFFFFF, None


def _map_bits(opt_map):
    m = int.from_bytes(bytes(bytearray(opt_map)), "little")
    k = 0
    while m:
        if m & 1:
            yield k
        m >>= 1
        k += 1


def IPv4OptionsFromMap(pkt, start, hlen, opt_map):
    """IPv4.Options and IPv4.Padding (ip4.go:219-256) of the header at
    pkt[start:start+hlen] from its gpk_fields option map (include/gpk.h: bit k
    = an option at header byte 20 + k), reading only the option bytes."""
    opts, padding = [], None
    for k in _map_bits(opt_map):
        b = start + 20 + k
        t = pkt[b]
        if t == 0:
            opts.append(IPv4Option(0, 1))
            padding = pkt[b + 1:start + hlen]
            break
        if t == 1:
            opts.append(IPv4Option(1, 1))
            continue
        ol = pkt[b + 1]
        opts.append(IPv4Option(t, ol, pkt[b + 2:b + ol]))
    return opts, padding


def hbh_map_covers(pkt, hbh_start):
    """Whether a gpk_fields hbh_opt_map holds the HopByHop header at
    pkt[hbh_start]: HeaderLength <= 2 (include/gpk.h)."""
    return pkt[hbh_start + 1] <= 2


def HopByHopFromMap(h, pkt, b0, e, opt_map):
    """IPv6HopByHop (ip6.go:418-432 base, :509-526 options, TLVs :327-346) of
    the header at pkt[b0] inside the IPv6 slice ending at e, from its
    gpk_fields option map: NextHeader and HeaderLength are the header's two
    bytes, each option read at its start."""
    h.NextHeader, h.HeaderLength = pkt[b0], pkt[b0 + 1]
    h.ActualLength = h.HeaderLength * 8 + 8
    h.Contents, h.Payload = pkt[b0:b0 + h.ActualLength], pkt[b0 + h.ActualLength:e]
    h.Options = []
    for k in _map_bits(opt_map):
        b = b0 + 2 + k
        if pkt[b] == 0:  # Pad1
            h.Options.append(IPv6HopByHopOption(0, 0, 1, None))
        else:
            al = pkt[b + 1] + 2
            h.Options.append(IPv6HopByHopOption(pkt[b], pkt[b + 1], al, pkt[b + 2:b + al]))
    return h


def _hbh_jumbo(pkt, b0, opt_map):
    """The jumbogram length of the HopByHop header at pkt[b0] (ip6.go:54-76:
    the first option of type 0xC2), or None."""
    for k in _map_bits(opt_map):
        b = b0 + 2 + k
        if pkt[b] == IPv6HopByHopOptionJumbogram:
            return _be32(pkt, b + 2)
    return None


def ipv6_payload_start(pkt, s, f):
    """Where the IPv6 layer at pkt[s]'s Payload starts (ip6.go:235-262): after
    the 40-byte header, and after an inline HopByHop header unless it is a
    jumbogram (P4: its payload is not advanced past the HopByHop header)."""
    if int(f["ip6_next_header"]) != IPProtocolIPv6HopByHop:
        return s + 40
    if int(f["ip6_length"]) == 0 and _hbh_jumbo(pkt, s + 40, f["hbh_opt_map"]) is not None:
        return s + 40
    return s + 40 + pkt[s + 41] * 8 + 8


def payload_end(kind, pkt, s, e, f):
    """The end of the Payload of the decoder `kind` whose DecodeFromBytes was
    handed pkt[s:e], from its gpk_fields values (each decoder's trim rule)."""
    if kind == _lib.DEC_ETHERNET:  # ethernet.go:50-55: 802.3 length trims, never grows
        return s + 14 + int(f["eth_length"]) if int(f["eth_type"]) == 0 and e - s - 14 > int(f["eth_length"]) else e
    if kind == _lib.DEC_IPV4:  # ip4.go:189-205 (Length already the slice's uint16 length when 0, P9)
        return s + int(f["ip4_length"]) if e - s > int(f["ip4_length"]) else e
    if kind == _lib.DEC_IPV6:  # ip6.go:244-277 (P3 / P4)
        p0, length = ipv6_payload_start(pkt, s, f), int(f["ip6_length"])
        if int(f["ip6_next_header"]) == IPProtocolIPv6HopByHop and length == 0:
            length = _hbh_jumbo(pkt, s + 40, f["hbh_opt_map"])
        return min(e, p0 + length) if p0 <= e else p0
    if kind == _lib.DEC_UDP:  # udp.go:46-55
        ln = int(f["udp_length"])
        return s + min(ln, e - s) if ln >= 8 else e
    return e


# ---- layers/ip6.go:434-461 ---------------------------------------------------
class IPv6ExtensionSkipper(BaseLayer):
    kind = _lib.DEC_IPV6_EXT

    def __init__(self):
        self.NextHeader = 0

    def CanDecode(self):
        return LayerClassIPv6Extension

    def NextLayerType(self):
        """ip6.go:458-461"""
        return IPProtocolLayerType(self.NextHeader)

    def _hydrate(self, d):
        actual = d[1] * 8 + 8
        self.NextHeader = d[0]
        self.Contents, self.Payload = d[:actual], d[actual:]
        self._poff = actual

    def _fill(self, pkt, s, e, f):
        # no record fields: NextHeader and HeaderLength are the header's first two bytes (ip6.go:418-461)
        actual = pkt[s + 1] * 8 + 8
        self.NextHeader = pkt[s]
        self.Contents, self.Payload = pkt[s:s + actual], pkt[s + actual:e]
        self._poff = actual


TCPOptionKindEndList, TCPOptionKindNop, TCPOptionKindMSS, TCPOptionKindTimestamps = 0, 1, 2, 8
TCPOptionKindMultipathTCP = 30
_TCP_OPTION_NAMES = {0: "EndList", 1: "NOP", 2: "MSS", 3: "WindowScale", 4: "SACKPermitted", 5: "SACK", 6: "Echo",
                     7: "EchoReply", 8: "Timestamps", 9: "PartialOrderConnectionPermitted",
                     10: "PartialOrderServiceProfile", 11: "CC", 12: "CCNew", 13: "CCEcho", 14: "AltChecksum",
                     15: "AltChecksumData", 30: "MultipathTCP"}  # tcp.go:62-101


def TCPOptionKindString(k):
    return _TCP_OPTION_NAMES.get(int(k), "Unknown(%d)" % int(k))


# ---- layers/multipathtcp.go: MPTCP option subtypes and their structs -----------
(MPTCPSubtypeMPCAPABLE, MPTCPSubtypeMPJOIN, MPTCPSubtypeDSS, MPTCPSubtypeADDADDR, MPTCPSubtypeREMOVEADDR,
 MPTCPSubtypeMPPRIO, MPTCPSubtypeMPFAIL, MPTCPSubtypeMPFASTCLOSE, MPTCPSubtypeMPTCPRST) = range(9)
_MPTCP_NAMES = ["MP_CAPABLE", "MP_JOIN", "DSS", "ADD_ADDR", "REMOVE_ADDR", "MP_PRIO", "MP_FAIL", "MP_FASTCLOSE",
                "MP_TCPRST"]


def MPTCPSubtypeString(k):
    return _MPTCP_NAMES[k] if 0 <= int(k) < len(_MPTCP_NAMES) else "Unknown(%d)" % int(k)


@dataclass
class MPCapable:
    Version: int = 0
    A: bool = False
    B: bool = False
    C: bool = False
    D: bool = False
    E: bool = False
    F: bool = False
    G: bool = False
    H: bool = False
    SendKey: Optional[bytes] = None
    ReceivKey: Optional[bytes] = None
    DataLength: int = 0
    Checksum: int = 0


@dataclass
class MPJoin:
    Backup: bool = False
    AddrID: int = 0
    ReceivToken: int = 0
    SendRandNum: int = 0
    SendHMAC: Optional[bytes] = None


@dataclass
class Dss:
    F: bool = False
    m: bool = False
    M: bool = False
    a: bool = False
    A: bool = False
    DataAck: Optional[bytes] = None
    DSN: Optional[bytes] = None
    SSN: int = 0
    DataLength: int = 0
    Checksum: int = 0


@dataclass
class AddAddr:
    IPVer: int = 0
    E: bool = False
    AddrID: int = 0
    Address: Optional[bytes] = None
    Port: int = 0
    SendHMAC: Optional[bytes] = None


@dataclass
class RemAddr:
    AddrIDs: Optional[list] = None


@dataclass
class MPPrio:
    Backup: bool = False
    AddrID: int = 0


@dataclass
class MPFail:
    DSN: int = 0


@dataclass
class MPFClose:
    ReceivKey: Optional[bytes] = None


@dataclass
class MPTcpRst:
    U: bool = False
    V: bool = False
    W: bool = False
    T: bool = False
    Reason: int = 0


@dataclass
class TCPOption:
    """tcp.go:103-117"""
    OptionType: int = 0
    OptionLength: int = 0
    OptionData: Optional[bytes] = None
    OptionMultipath: int = 0
    OptionMPTCPMpCapable: Optional[MPCapable] = None
    OptionMPTCPDss: Optional[Dss] = None
    OptionMPTCPMpJoin: Optional[MPJoin] = None
    OptionMPTCPMpPrio: Optional[MPPrio] = None
    OptionMPTCPAddAddr: Optional[AddAddr] = None
    OptionMTCPRemAddr: Optional[RemAddr] = None
    OptionMTCPMPFastClose: Optional[MPFClose] = None
    OptionMPTCPMPTcpRst: Optional[MPTcpRst] = None
    OptionMTCPMPFail: Optional[MPFail] = None

    def String(self):
        """tcp.go:120-184"""
        d = self.OptionData or b""
        hd = (" 0x" + d.hex()) if d else ""
        k = TCPOptionKindString(self.OptionType)
        if self.OptionType == TCPOptionKindMSS and len(d) >= 2:
            return "TCPOption(%s:%d%s)" % (k, _be16(d, 0), hd)
        if self.OptionType == TCPOptionKindTimestamps and len(d) == 8:
            return "TCPOption(%s:%d/%d%s)" % (k, _be32(d, 0), _be32(d, 4), hd)
        if self.OptionType == TCPOptionKindMultipathTCP:
            st, n, gb = self.OptionMultipath, MPTCPSubtypeString(self.OptionMultipath), lambda b: str(b).lower()
            if st == MPTCPSubtypeMPCAPABLE:
                return "MPTCPOption(%s Version %d)" % (n, self.OptionMPTCPMpCapable.Version)
            if st == MPTCPSubtypeMPJOIN:
                j = self.OptionMPTCPMpJoin
                return "MPTCPOption(%s Backup %s;Address ID %d)" % (n, gb(j.Backup), j.AddrID)
            if st in (MPTCPSubtypeDSS, MPTCPSubtypeMPFASTCLOSE, MPTCPSubtypeMPFAIL):
                return "MPTCPOption(%s)" % n
            if st == MPTCPSubtypeMPPRIO:
                q = self.OptionMPTCPMpPrio
                return "MPTCPOption(%s Backup %s;Address ID %d)" % (n, gb(q.Backup), q.AddrID)
            if st == MPTCPSubtypeADDADDR:
                a = self.OptionMPTCPAddAddr
                from .gopacket import _ip_string
                return "MPTCPOption(%s Address ID %d;Address %s;Port %d)" % (n, a.AddrID, _ip_string(a.Address or b""),
                                                                           a.Port)
            if st == MPTCPSubtypeREMOVEADDR:
                return "MPTCPOption(%s Address ID [%s])" % (n, " ".join(str(x) for x in self.OptionMTCPRemAddr.AddrIDs))
            if st == MPTCPSubtypeMPTCPRST:
                r = self.OptionMPTCPMPTcpRst
                return "MPTCPOption(%s Transient %s; Reason %d)" % (n, gb(r.T), r.Reason)
        return "TCPOption(%s:%s)" % (k, hd)

    __str__ = String


def _mptcp_option(o, d):
    """The MPTCP option struct tcp.go:346-527 builds from the option at d[0]
    (d: the rest of the options area; the packet decoded without error, so its
    lengths are ones the reference accepts)."""
    L, st = o.OptionLength, o.OptionMultipath
    b16 = lambda a: _be16(d, a)  # noqa: E731
    b32 = lambda a: _be32(d, a)  # noqa: E731
    if st == MPTCPSubtypeMPCAPABLE:
        f = d[3]
        c = MPCapable(d[2] & 0x0F, *(bool(f & (0x80 >> i)) for i in range(8)))
        if L >= 12:
            c.SendKey = bytes(d[4:12])
        if L >= 20:
            c.ReceivKey = bytes(d[12:20])
        if L >= 22:
            c.DataLength = b16(20)
        if L == 24:
            c.Checksum = b16(22)
        o.OptionMPTCPMpCapable = c
    elif st == MPTCPSubtypeMPJOIN:
        if L == 12:
            o.OptionMPTCPMpJoin = MPJoin(bool(d[2] & 1), d[3], b32(4), b32(8))
        elif L == 16:
            o.OptionMPTCPMpJoin = MPJoin(bool(d[2] & 1), d[3], SendHMAC=bytes(d[4:12]), SendRandNum=b32(12))
        elif L == 24:
            o.OptionMPTCPMpJoin = MPJoin(SendHMAC=bytes(d[4:24]))
    elif st == MPTCPSubtypeDSS:
        f = d[3]
        x = Dss(bool(f & 0x10), bool(f & 0x08), bool(f & 0x04), bool(f & 0x02), bool(f & 0x01))
        k = 4
        if x.A:
            n = 8 if x.a else 4
            x.DataAck, k = bytes(d[k:k + n]), k + n
        if x.M:
            n = 8 if x.m else 4
            x.DSN, k = bytes(d[k:k + n]), k + n
            x.SSN, k = b32(k), k + 4
            x.DataLength, k = b16(k), k + 2
            if (L - k) & 0xFF == 2:
                x.Checksum = b16(k)
        o.OptionMPTCPDss = x
    elif st == MPTCPSubtypeADDADDR:
        n = L
        if d[2] & 0x0F > 1:
            a = AddAddr(IPVer=d[2] & 0x0F, AddrID=d[3])
        else:
            a = AddAddr(E=bool(d[2] & 1), AddrID=d[3])
            if not a.E:
                a.SendHMAC = bytes(d[L - 8:])  # to the end of the options area, as Go's data[L-8:]
                n = (n - 8) & 0xFF
        if n in (8, 10):
            a.Address = bytes(d[4:8])
        elif n in (20, 22):
            a.Address = bytes(d[4:20])
        if n == 10:
            a.Port = b16(8)
        elif n == 22:
            a.Port = b16(20)
        o.OptionMPTCPAddAddr = a
    elif st == MPTCPSubtypeREMOVEADDR:
        o.OptionMTCPRemAddr = RemAddr(list(d[3:3 + (L - 3)]))
    elif st == MPTCPSubtypeMPPRIO:
        o.OptionMPTCPMpPrio = MPPrio(bool(d[2] & 1), d[3] if L == 4 else 0)
    elif st == MPTCPSubtypeMPFAIL:
        o.OptionMTCPMPFail = MPFail(struct.unpack(">Q", bytes(d[4:12]))[0])
    elif st == MPTCPSubtypeMPFASTCLOSE:
        o.OptionMTCPMPFastClose = MPFClose(bytes(d[4:12]))
    elif st == MPTCPSubtypeMPTCPRST:
        o.OptionMPTCPMPTcpRst = MPTcpRst(bool(d[2] & 8), bool(d[2] & 4), bool(d[2] & 2), bool(d[2] & 1), d[3])
    return o


# ---- layers/tcp.go:19-551 ----------------------------------------------------
class TCP(BaseLayer, _Checksummed):
    kind = _lib.DEC_TCP

    def __init__(self):
        self.SrcPort = self.DstPort = 0
        self.Seq = self.Ack = 0
        self.DataOffset = 0
        self.FIN = self.SYN = self.RST = self.PSH = self.ACK = self.URG = self.ECE = self.CWR = self.NS = False
        self.Window = self.Checksum = self.Urgent = 0
        self.Options: List[TCPOption] = []
        self.Padding = b""
        self.Multipath = False
        self.sPort = self.dPort = b""

    def LayerType(self):
        return LayerTypeTCP

    def CanDecode(self):
        return LayerClass([LayerTypeTCP])

    def _hydrate(self, d):
        self.SrcPort, self.DstPort = _be16(d, 0), _be16(d, 2)
        self.sPort, self.dPort = d[0:2], d[2:4]
        self.Seq, self.Ack = _be32(d, 4), _be32(d, 8)
        self.DataOffset = d[12] >> 4
        f = d[13]
        self.FIN, self.SYN, self.RST, self.PSH = bool(f & 1), bool(f & 2), bool(f & 4), bool(f & 8)
        self.ACK, self.URG, self.ECE, self.CWR = bool(f & 0x10), bool(f & 0x20), bool(f & 0x40), bool(f & 0x80)
        self.NS = bool(d[12] & 1)
        self.Window, self.Checksum, self.Urgent = _be16(d, 14), _be16(d, 16), _be16(d, 18)
        ds = self.DataOffset * 4
        self.Contents, self.Payload = d[:ds], d[ds:]
        self.Options, self.Padding = [], b""
        opts = d[20:ds]
        while len(opts) > 0:
            t = opts[0]
            if t == 0:
                self.Options.append(TCPOption(0, 1))
                self.Padding = opts[1:]
                break
            if t == 1:
                o = TCPOption(1, 1)
            elif t == TCPOptionKindMultipathTCP:
                self.Multipath = True
                o = _mptcp_option(TCPOption(t, opts[1], None, opts[2] >> 4), opts)
            else:
                o = TCPOption(t, opts[1], opts[2:opts[1]])
            self.Options.append(o)
            opts = opts[o.OptionLength:]
        self._poff = ds

    def _fill(self, pkt, s, e, f):
        self.SrcPort, self.DstPort = int(f["tcp_src_port"]), int(f["tcp_dst_port"])
        self.sPort, self.dPort = struct.pack(">H", self.SrcPort), struct.pack(">H", self.DstPort)
        self.Seq, self.Ack, self.DataOffset = int(f["tcp_seq"]), int(f["tcp_ack"]), int(f["tcp_data_offset"])
        fl = int(f["tcp_flags"])
        self.FIN, self.SYN, self.RST, self.PSH = bool(fl & 1), bool(fl & 2), bool(fl & 4), bool(fl & 8)
        self.ACK, self.URG, self.ECE, self.CWR = bool(fl & 0x10), bool(fl & 0x20), bool(fl & 0x40), bool(fl & 0x80)
        self.NS = bool(fl & 0x100)
        self.Window, self.Checksum, self.Urgent = int(f["tcp_window"]), int(f["tcp_checksum"]), int(f["tcp_urgent"])
        ds = self.DataOffset * 4
        self.Contents, self.Payload = pkt[s:s + ds], pkt[s + ds:e]
        self.Options, self.Padding, mp = TCPOptionsFromMap(pkt, s, ds, f["tcp_opt_map"])
        if mp:  # tcp.go:348: set by an MPTCP option, never reset (P6)
            self.Multipath = True
        self._poff = ds

    def NextLayerType(self):
        """tcp.go:591-597: the destination port's type, else the source port's"""
        lt = TCPPortLayerType(self.DstPort)
        return TCPPortLayerType(self.SrcPort) if lt == LayerTypePayload else lt

    def TransportFlow(self):
        return NewFlow(EndpointTCPPort, self.sPort, self.dPort)

    def ComputeChecksum(self):
        """tcp.go:251-257: (uint16, error) over Contents + Payload as they are
        (the header's own Checksum field included: 0 for a correct segment)."""
        from .gopacket import FoldChecksum
        csum, err = self._compute_checksum(bytes(self.Contents) + bytes(self.Payload), 6)
        return (0, err) if err is not None else (FoldChecksum(csum), None)


def TCPOptionsFromMap(pkt, start, hlen, opt_map):
    """TCP.Options, TCP.Padding and TCP.Multipath (tcp.go:336-549) of the
    header at pkt[start:start+hlen] from its gpk_fields option map."""
    opts, padding, mp = [], b"", False
    for k in _map_bits(opt_map):
        b = start + 20 + k
        t = pkt[b]
        if t == 0:
            opts.append(TCPOption(0, 1))
            padding = pkt[b + 1:start + hlen]
            break
        if t == 1:
            opts.append(TCPOption(1, 1))
        elif t == TCPOptionKindMultipathTCP:
            mp = True
            opts.append(_mptcp_option(TCPOption(t, pkt[b + 1], None, pkt[b + 2] >> 4), pkt[b:start + hlen]))
        else:
            opts.append(TCPOption(t, pkt[b + 1], pkt[b + 2:b + pkt[b + 1]]))
    return opts, padding, mp


# ---- layers/udp.go:17-56 -----------------------------------------------------
class UDP(BaseLayer, _Checksummed):
    kind = _lib.DEC_UDP

    def __init__(self):
        self.SrcPort = self.DstPort = self.Length = self.Checksum = 0
        self.sPort = self.dPort = b""

    def LayerType(self):
        return LayerTypeUDP

    def CanDecode(self):
        return LayerClass([LayerTypeUDP])

    def _hydrate(self, d):
        self.SrcPort, self.DstPort = _be16(d, 0), _be16(d, 2)
        self.sPort, self.dPort = d[0:2], d[2:4]
        self.Length, self.Checksum = _be16(d, 4), _be16(d, 6)
        self.Contents = d[:8]
        if self.Length >= 8:
            self.Payload = d[8:min(self.Length, len(d))]
        else:
            self.Payload = d[8:]
        self._poff = 8

    def _fill(self, pkt, s, e, f):
        self.SrcPort, self.DstPort = int(f["udp_src_port"]), int(f["udp_dst_port"])
        self.sPort, self.dPort = struct.pack(">H", self.SrcPort), struct.pack(">H", self.DstPort)
        self.Length, self.Checksum = int(f["udp_length"]), int(f["udp_checksum"])
        self.Contents, self.Payload = pkt[s:s + 8], pkt[s + 8:payload_end(_lib.DEC_UDP, pkt, s, e, f)]
        self._poff = 8

    def NextLayerType(self):
        """udp.go:114-119"""
        lt = UDPPortLayerType(self.DstPort)
        return lt if lt != LayerTypePayload else UDPPortLayerType(self.SrcPort)

    def TransportFlow(self):
        return NewFlow(EndpointUDPPort, self.sPort, self.dPort)


__all__ = [n for n in dir() if not n.startswith("_")]


# ---- endpoints (layers/endpoints.go:51-99) --------------------------------------


def _to4(ip):  # net.IP.To4
    if len(ip) == 4:
        return ip
    if len(ip) == 16 and ip[:10] == bytes(10) and ip[10:12] == b"\xff\xff":
        return ip[12:]
    return None


def NewIPEndpoint(ip):
    """An IPv4 endpoint for a 4-byte or IPv4-mapped address, IPv6 for another
    16-byte one, InvalidEndpoint otherwise (ip: bytes or an ipaddress object)."""
    b = ip.packed if hasattr(ip, "packed") else bytes(ip)
    v4 = _to4(b)
    if v4 is not None:
        return NewEndpoint(EndpointIPv4, v4)
    if len(b) == 16:
        return NewEndpoint(EndpointIPv6, b)
    return InvalidEndpoint


def NewMACEndpoint(mac):
    return NewEndpoint(EndpointMAC, bytes(mac))


def _port_endpoint(t, p):
    return NewEndpoint(t, bytes([(p >> 8) & 0xFF, p & 0xFF]))


def NewTCPPortEndpoint(p):
    return _port_endpoint(EndpointTCPPort, int(p))


def NewUDPPortEndpoint(p):
    return _port_endpoint(EndpointUDPPort, int(p))


def NewSCTPPortEndpoint(p):
    return _port_endpoint(EndpointSCTPPort, int(p))


def NewRUDPPortEndpoint(p):
    return NewEndpoint(EndpointRUDPPort, bytes([int(p) & 0xFF]))


def NewUDPLitePortEndpoint(p):
    return _port_endpoint(EndpointUDPLitePort, int(p))
