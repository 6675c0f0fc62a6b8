"""The gopacket root-package surface of the hot path, over the device engine.

Mirrors (reference file:line):
  LayerType / LayerTypeZero.. (layertype.go:20-111, decode.go:106-117)
  Endpoint, Flow, NewFlow, NewEndpoint, FlowFromEndpoints, LessThan, FastHash,
  RegisterEndpointType / EndpointType names (flows.go:27-236, layers/endpoints.go:17-49)
  ChecksumVerificationResult, ComputeChecksum, FoldChecksum (checksum.go:14-58)
  RegisterLayerType / OverrideLayerType / LayerTypeMetadata (layertype.go:22-83)
  LayerClassSlice / LayerClassMap / NewLayerClass (layerclass.go:9-107)
  Payload, Fragment DecodingLayers (base.go:40-124)
  DecodingLayerParser, NewDecodingLayerParser, DecodeLayers, AddDecodingLayer,
  UnsupportedLayerType, DecodingLayerParserOptions (parser.go:182-351)

Decoding always runs on the GPU (through include/gpk.h): DecodeLayers sends
one packet, DecodeBatch a whole PacketBatch; the per-packet results fill the
registered layer structs exactly as the reference's DecodeLayers would.
"""
import json
import os
import struct
from dataclasses import dataclass

import numpy as np

from . import _lib

_REG = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "registry_gen.json")))
_LT_NAMES = {int(k): v for k, v in _REG["layer_type_names"].items()}


class LayerType(int):
    """gopacket.LayerType (layertype.go:20); String() per layertype.go:101-111;
    a LayerType is a LayerClass of itself (layerclass.go:21-29)."""

    def String(self):
        s = _LT_NAMES.get(int(self), "")
        return s if s else str(int(self))

    __str__ = String

    def __repr__(self):
        return "LayerType(%s)" % self.String()

    def Contains(self, a):
        return int(self) == int(a)

    def LayerTypes(self):
        return [self]


@dataclass
class LayerTypeMetadata:  # layertype.go:22-29 (Decoder: the NewPacket path, outside the hot path)
    Name: str
    Decoder: object = None


DecodersByLayerName = {}  # layertype.go:39
_LT_IN_USE = set(_LT_NAMES)


def RegisterLayerType(num, meta):
    """layertype.go:53-64: a new layer type (panics when the number is taken).
    Its name is what String(), UnsupportedLayerType and the decoded lists print."""
    if int(num) in _LT_IN_USE:
        raise GoPanic("Layer type already exists")
    return OverrideLayerType(num, meta)


def OverrideLayerType(num, meta):
    """layertype.go:69-83"""
    _LT_IN_USE.add(int(num))
    _LT_NAMES[int(num)] = meta.Name
    DecodersByLayerName[meta.Name] = meta.Decoder
    return LayerType(num)


class LayerClass(list):
    """layerclass.go:11-107: the LayerTypes a DecodingLayer can decode
    (CanDecode); a single LayerType or a LayerClassSlice in Go."""

    def Contains(self, t):
        return int(t) in [int(x) for x in self]

    def LayerTypes(self):
        return list(self)


class LayerClassSlice(list):
    """layerclass.go:31-67: a []bool indexed by LayerType."""

    def Contains(self, t):
        return 0 <= int(t) < len(self) and bool(self[int(t)])

    def LayerTypes(self):
        return [LayerType(i) for i, v in enumerate(self) if v]


class LayerClassMap(dict):
    """layerclass.go:69-94: a map[LayerType]bool."""

    def Contains(self, t):
        return bool(self.get(int(t), False))

    def LayerTypes(self):
        return [LayerType(t) for t in self]


def NewLayerClassSlice(types):
    m = max([0] + [int(t) for t in types])
    s = LayerClassSlice([False] * (m + 1))
    for t in types:
        s[int(t)] = True
    return s


def NewLayerClassMap(types):
    return LayerClassMap({int(t): True for t in types})


def NewLayerClass(types):
    """layerclass.go:98-107: a map when any type exceeds maxLayerType (2000), else a slice."""
    if any(int(t) > 2000 for t in types):
        return NewLayerClassMap(types)
    return NewLayerClassSlice(types)


LayerTypeZero = LayerType(0)
LayerTypeDecodeFailure = LayerType(1)
LayerTypePayload = LayerType(2)
LayerTypeFragment = LayerType(3)

# ---- errors ----------------------------------------------------------------


class GoError:
    """An `error` value returned by DecodeLayers (compare with Error())."""

    def __init__(self, msg):
        self.msg = msg

    def Error(self):
        return self.msg

    __str__ = Error

    def __repr__(self):
        return "GoError(%r)" % self.msg

    def __eq__(self, other):
        return isinstance(other, GoError) and other.Error() == self.Error()


class UnsupportedLayerType(GoError):
    """parser.go:319-327"""

    def __init__(self, typ):
        self.typ = LayerType(typ)
        super().__init__("No decoder for layer type %s" % self.typ.String())


class GoPanic(RuntimeError):
    """A decoder panic with IgnorePanic set: the reference lets it propagate."""


# ---- checksum / flows ------------------------------------------------------


@dataclass
class ChecksumVerificationResult:
    Valid: bool = False
    Correct: int = 0
    Actual: int = 0


def ComputeChecksum(data, csum=0):
    """checksum.go:35-50: RFC 1071 sum of big-endian 16-bit words (an odd last
    byte as the high byte) added to csum, in uint32 arithmetic (it wraps)."""
    b = np.frombuffer(bytes(data), np.uint8)
    n = len(b) & ~1
    w = b[:n].reshape(-1, 2).astype(np.uint64)
    total = int(csum) + int((w[:, 0] << 8).sum() + w[:, 1].sum())
    if len(b) & 1:
        total += int(b[-1]) << 8
    return total & 0xFFFFFFFF


def FoldChecksum(csum):
    """checksum.go:53-58"""
    csum &= 0xFFFFFFFF
    while csum > 0xFFFF:
        csum = (csum >> 16) + (csum & 0xFFFF)
    return ~csum & 0xFFFF


MaxEndpointSize = 16
_FNV_BASIS = 14695981039346656037
_FNV_PRIME = 1099511628211
_M64 = (1 << 64) - 1


def _fnv(b):
    h = _FNV_BASIS
    for x in b:
        h = ((h ^ x) * _FNV_PRIME) & _M64
    return h


def _go_bytes(b):  # fmt's %v of a []byte / [N]byte: "[1 2 3]"
    return "[" + " ".join(str(x) for x in b) + "]"


def _ip_string(b):
    """net.IP.String (Go): dotted for 4 bytes and IPv4-mapped 16, RFC 5952 for IPv6."""
    import ipaddress
    if len(b) == 0:
        return "<nil>"
    if len(b) == 4:
        return str(ipaddress.IPv4Address(bytes(b)))
    if len(b) == 16:
        if b[:10] == bytes(10) and b[10:12] == b"\xff\xff":
            return str(ipaddress.IPv4Address(bytes(b[12:])))
        return ipaddress.IPv6Address(bytes(b)).compressed
    return "?" + bytes(b).hex()


@dataclass
class EndpointTypeMetadata:  # flows.go:99-106
    Name: str
    Formatter: object = None  # bytes -> str


_endpoint_types = {}


class EndpointType(int):
    """flows.go:108-131: registered types print their name, others their number."""

    def String(self):
        m = _endpoint_types.get(int(self))
        return m.Name if m is not None else str(int(self))

    __str__ = String


def RegisterEndpointType(num, meta):
    """flows.go:117-124 (panics on a number already in use)."""
    if num in _endpoint_types:
        raise GoPanic("Endpoint type number already in use")
    _endpoint_types[num] = meta
    return EndpointType(num)


def _port(b):
    if len(b) < 2:  # binary.BigEndian.Uint16: _ = b[1]
        raise GoPanic("runtime error: index out of range [1] with length %d" % len(b))
    return str(struct.unpack(">H", bytes(b[:2]))[0])


EndpointInvalid = RegisterEndpointType(0, EndpointTypeMetadata("invalid", _go_bytes))  # flows.go:228-230
# layers/endpoints.go:21-48
EndpointIPv4 = RegisterEndpointType(1, EndpointTypeMetadata("IPv4", _ip_string))
EndpointIPv6 = RegisterEndpointType(2, EndpointTypeMetadata("IPv6", _ip_string))
EndpointMAC = RegisterEndpointType(3, EndpointTypeMetadata("MAC", lambda b: ":".join("%02x" % x for x in b)))
EndpointTCPPort = RegisterEndpointType(4, EndpointTypeMetadata("TCP", _port))
EndpointUDPPort = RegisterEndpointType(5, EndpointTypeMetadata("UDP", _port))
EndpointSCTPPort = RegisterEndpointType(6, EndpointTypeMetadata("SCTP", _port))
EndpointRUDPPort = RegisterEndpointType(7, EndpointTypeMetadata("RUDP", lambda b: str(b[0])))
EndpointUDPLitePort = RegisterEndpointType(8, EndpointTypeMetadata("UDPLite", _port))
EndpointPPP = RegisterEndpointType(9, EndpointTypeMetadata("PPP", lambda b: "point"))


class Endpoint:
    """flows.go:32-97, 133-138"""

    def __init__(self, typ, raw):
        if len(raw) > MaxEndpointSize:
            raise GoPanic("raw byte length greater than MaxEndpointSize")
        self.typ, self.raw = EndpointType(typ), bytes(raw)

    def EndpointType(self):
        return self.typ

    def Raw(self):
        return self.raw

    def LessThan(self, b):  # flows.go:53-55
        return self.typ < b.typ or (self.typ == b.typ and self.raw < b.raw)

    def FastHash(self):
        return ((_fnv(self.raw) ^ self.typ) * _FNV_PRIME) & _M64

    def __eq__(self, o):
        return isinstance(o, Endpoint) and (self.typ, self.raw) == (o.typ, o.raw)

    def __hash__(self):
        return hash((self.typ, self.raw))

    def String(self):
        m = _endpoint_types.get(int(self.typ))
        if m is not None and m.Formatter is not None:
            return m.Formatter(self.raw)
        return "%s:%s" % (self.typ.String(), _go_bytes(self.raw.ljust(MaxEndpointSize, b"\x00")))  # %v of the [16]byte

    __str__ = String


def NewEndpoint(typ, raw):
    """flows.go:89-97"""
    return Endpoint(typ, raw)


class Flow:
    """flows.go:142-224. FastHash() of a Flow taken from a decoded packet is
    the hash the device computed; a Flow built by hand hashes on the host."""

    def __init__(self, typ, src, dst, fast_hash=None):
        if len(src) > MaxEndpointSize or len(dst) > MaxEndpointSize:
            raise GoPanic("flow raw byte length greater than MaxEndpointSize")
        self.typ, self.src, self.dst = EndpointType(typ), bytes(src), bytes(dst)
        self._hash = fast_hash

    def FastHash(self):
        if self._hash is not None:
            return self._hash
        return (((_fnv(self.src) + _fnv(self.dst)) & _M64) ^ self.typ) * _FNV_PRIME & _M64

    def EndpointType(self):
        return self.typ

    def Endpoints(self):
        return Endpoint(self.typ, self.src), Endpoint(self.typ, self.dst)

    def Src(self):
        return Endpoint(self.typ, self.src)

    def Dst(self):
        return Endpoint(self.typ, self.dst)

    def Reverse(self):
        return Flow(self.typ, self.dst, self.src, self._hash)  # FastHash is symmetric

    def __eq__(self, o):
        return isinstance(o, Flow) and (self.typ, self.src, self.dst) == (o.typ, o.src, o.dst)

    def __hash__(self):
        return hash((self.typ, self.src, self.dst))

    def String(self):
        return "%s->%s" % (self.Src(), self.Dst())

    __str__ = String


def NewFlow(t, src, dst):
    return Flow(t, src, dst)


def FlowFromEndpoints(src, dst):
    """flows.go:151-157: (Flow, None), or (the zero Flow, error) for mismatched types."""
    if src.typ != dst.typ:
        return Flow(0, b"", b""), GoError("Mismatched endpoint types: %s->%s" % (src.typ.String(), dst.typ.String()))
    return Flow(src.typ, src.raw, dst.raw), None


InvalidEndpoint = NewEndpoint(EndpointInvalid, b"")  # flows.go:233
InvalidFlow = NewFlow(EndpointInvalid, b"", b"")      # flows.go:236


# ---- Payload / Fragment ----------------------------------------------------


class Payload:
    """base.go:40-70"""
    kind = _lib.DEC_PAYLOAD

    def __init__(self):
        self.data = b""

    def CanDecode(self):
        return LayerClass([LayerTypePayload])

    def LayerType(self):
        return LayerTypePayload

    def NextLayerType(self):
        return LayerTypeZero

    def LayerContents(self):
        return self.data

    def LayerPayload(self):
        return b""

    def Payload(self):
        return self.data

    def _hydrate(self, d):
        self.data = d
        self._poff = len(d)

    def _fill(self, pkt, s, e, f):
        self._hydrate(pkt[s:e])


class Fragment(Payload):
    """base.go:95-124"""
    kind = _lib.DEC_FRAGMENT

    def CanDecode(self):
        return LayerClass([LayerTypeFragment])

    def LayerType(self):
        return LayerTypeFragment


# ---- packet batches ------------------------------------------------------------


class PacketBatch:
    """A packed, offset-indexed host batch (the gpk_batch layout)."""

    def __init__(self, data, offsets, caplens):
        self.data = np.ascontiguousarray(data, dtype=np.uint8)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.caplens = np.ascontiguousarray(caplens, dtype=np.uint32)

    @classmethod
    def from_packets(cls, packets):
        packets = [bytes(p) for p in packets]
        caplens = np.array([len(p) for p in packets], np.uint32)
        offsets = np.zeros(len(packets), np.uint64)
        if len(packets) > 1:
            offsets[1:] = np.cumsum(caplens[:-1], dtype=np.uint64)
        return cls(np.frombuffer(b"".join(packets) + bytes(16), np.uint8), offsets, caplens)

    def __len__(self):
        return len(self.offsets)

    def packet(self, i):
        o, c = int(self.offsets[i]), int(self.caplens[i])
        return bytes(self.data[o:o + c])


# ---- the parser ------------------------------------------------------------------

_DEFAULT_CTX = None


def _default_ctx():
    global _DEFAULT_CTX
    if _DEFAULT_CTX is None:
        from .engine import Context
        _DEFAULT_CTX = Context(int(os.environ.get("GPK_DEVICE", "0")))
    return _DEFAULT_CTX


# ---- decoding layer containers (parser.go:48-169) ------------------------------


class DecodingLayerContainer:
    """parser.go:56-67: LayerType -> DecodingLayer. Put registers every type of
    the layer's CanDecode() (a later Put overrides); Decoder looks one up;
    LayersDecoder returns the DecodingLayerFunc of the container. The three
    forms differ in their lookup structure only; the device decodes with
    the container's contents either way (layers_decoder.go:18-100)."""

    def LayersDecoder(self, first, df):
        """parser.go:96-99 / 138-141 / 166-169: a DecodingLayerFunc over this
        container starting at `first`, reporting Truncated to df."""
        return _LayersDecoder(self, LayerType(first), df)

    def _instances(self):
        """Each registered DecodingLayer once, by its device decoder kind
        (_types: the subclass's (LayerType, layer) pairs)."""
        out = {}
        for _, d in self._types():
            if d is not None:
                out[d.kind] = d
        return out


class DecodingLayerSparse(DecodingLayerContainer):
    """parser.go:74-107: a slice indexed by the LayerType value."""

    def __init__(self, layers=None):
        self._slots = list(layers or [])

    def Put(self, d):
        types = [int(t) for t in d.CanDecode().LayerTypes()]
        slots = self._slots + [None] * max(0, max(types) + 1 - len(self._slots))
        for t in types:
            slots[t] = d
        return DecodingLayerSparse(slots)

    def Decoder(self, typ):
        t = int(typ)
        d = self._slots[t] if 0 <= t < len(self._slots) else None
        return d, d is not None

    def _types(self):
        return [(t, d) for t, d in enumerate(self._slots) if d is not None]


class DecodingLayerArray(DecodingLayerContainer):
    """parser.go:112-142: (type, layer) pairs searched linearly."""

    def __init__(self, elems=None):
        self._elems = list(elems or [])

    def Put(self, d):
        elems = list(self._elems)
        for t in d.CanDecode().LayerTypes():
            for k, (typ, _) in enumerate(elems):
                if typ == int(t):
                    elems[k] = (typ, d)
                    break
            else:
                elems.append((int(t), d))
        return DecodingLayerArray(elems)

    def Decoder(self, typ):
        for t, d in self._elems:
            if t == int(typ):
                return d, True
        return None, False

    def _types(self):
        return list(self._elems)


class DecodingLayerMap(DecodingLayerContainer):
    """parser.go:147-169: a map keyed by LayerType (the parser's default)."""

    def __init__(self, m=None):
        self._m = dict(m or {})

    def Put(self, d):
        m = dict(self._m)
        for t in d.CanDecode().LayerTypes():
            m[int(t)] = d
        return DecodingLayerMap(m)

    def Decoder(self, typ):
        d = self._m.get(int(typ))
        return d, d is not None

    def _types(self):
        return list(self._m.items())


class _NilDecodeFeedback:
    """decode.go:21-26"""

    def SetTruncated(self):
        pass


NilDecodeFeedback = _NilDecodeFeedback()


class _LayersDecoder:
    """LayersDecoder (layers_decoder.go:11-101) for one packet on the device:
    returns (LayerTypeZero, None) on success, (the first LayerType with no
    decoder, None), or (LayerTypeZero, the decoder's error). A decoder's panic
    is not recovered here (DecodeLayers recovers it, parser.go:329-333): it
    raises GoPanic. `decoded` is truncated and refilled, except when `first`
    has no decoder (returned at once, layers_decoder.go:12-16)."""

    def __init__(self, dlc, first, df, overrides=None):
        self.dlc, self.first, self.df = dlc, first, df
        self._p = DecodingLayerParser(first)
        self._p.SetDecodingLayerContainer(dlc)
        self._p.IgnorePanic = True  # panics raise (GoPanic) instead of becoming errors
        self._p._overrides = overrides

    def __call__(self, data, decoded):
        if not self.dlc.Decoder(self.first)[1]:
            return self.first, None
        if self.df is not None and hasattr(self.df, "_ctx"):
            self._p._ctx = self._p._ctx or self.df._ctx
        res = self._p.DecodeBatch(PacketBatch.from_packets([data]), layouts=True)
        err = res.Hydrate(0, decoded)
        if res.Truncated(0) and self.df is not None:
            self.df.SetTruncated()
        if isinstance(err, UnsupportedLayerType):
            return err.typ, None
        return LayerTypeZero, err


class DecodingLayerParser:
    """parser.go:182-317 over the GPU engine.

    Differences that are not semantic: the device decodes the container's
    layers whichever container form holds them (Sparse/Array/Map decode
    identically, layers_decoder.go:18-100); layer structs are refreshed from
    device results, so per-packet state that the reference leaves stale
    across calls (TCP.Multipath, IPv4.Padding) is per packet here
    (parity notes P6)."""

    def __init__(self, first, *decoders, ctx=None):
        self.first = LayerType(first)
        self.IgnorePanic = False
        self.IgnoreUnsupported = False
        self.Truncated = False
        self._ctx = ctx
        self._overrides = None  # next-layer table entries of this parser alone (DecodeFromBytes)
        dlc = DecodingLayerMap()  # NewDecodingLayerParser's default container (parser.go:226)
        for d in decoders:
            dlc = dlc.Put(d)
        self.SetDecodingLayerContainer(dlc)

    def SetDecodingLayerContainer(self, dlc):
        """parser.go:238-241: replaces every registered decoder."""
        self._dlc = dlc
        self._decoders = dlc._instances()  # kind -> instance
        self._cfg = None

    def AddDecodingLayer(self, d):
        """parser.go:200-202"""
        self.SetDecodingLayerContainer(self._dlc.Put(d))

    def SetTruncated(self):
        """parser.go:207-209 (the parser is its decoders' DecodeFeedback)"""
        self.Truncated = True

    def _config(self, outputs=_lib.OUT_ALL):
        from .engine import ParserConfig
        from . import layers
        ed = layers._registry_edits()  # EthernetTypeMetadata / IPProtocolMetadata edits, Register*PortLayerType
        for k, v in (self._overrides or {}).items():
            ed[k] = list(ed[k]) + list(v)
        key = (tuple(sorted(self._decoders)), self.IgnorePanic, self.IgnoreUnsupported, outputs,
               tuple((k, tuple(v)) for k, v in sorted(ed.items())))
        if self._cfg is None or self._cfg[0] != key:
            p = ParserConfig(int(self.first), sorted(self._decoders), ignore_panic=self.IgnorePanic,
                             ignore_unsupported=self.IgnoreUnsupported, outputs=outputs)
            for v, lt in ed["ethertype"]:
                p.set_ethertype(v, lt)
            for v, lt in ed["ipprotocol"]:
                p.set_ipprotocol(v, lt)
            for v, lt in ed["tcp_port"]:
                p.set_tcp_port(v, lt)
            for v, lt in ed["udp_port"]:
                p.set_udp_port(v, lt)
            self._cfg = (key, p)
        return self._cfg[1]

    def ctx(self):
        return self._ctx or _default_ctx()

    def DecodeLayers(self, data, decoded):
        """Decode one packet on the GPU; fills the registered layers and the
        `decoded` list (truncated first, as parser.go:303-317 does)."""
        batch = PacketBatch.from_packets([data])
        res = self.DecodeBatch(batch, layouts=True)
        return res.Hydrate(0, decoded)

    def DecodeBatch(self, batch, layouts=False, outputs=_lib.OUT_ALL, fields=False):
        """DecodeLayers for every packet of the batch on the device. fields=True
        also returns each packet's scalar layer fields and IPv4/TCP option maps
        computed on the device (BatchResult.fields, FIELDS_DTYPE;
        BatchResult.IPv4Options / TCPOptions): in the decode launch itself
        (gpk_decode_batch_fields) when layouts=False, else from the layouts
        (gpk_extract_fields), which Hydrate needs."""
        cfg = self._config(outputs)
        if fields:
            r, f = self.ctx().decode_host_fields(cfg, batch.data, batch.offsets, batch.caplens, layouts=layouts)
            res = BatchResult(self, batch, r)
            res.fields = f
            return res
        r = self.ctx().decode_host(cfg, batch.data, batch.offsets, batch.caplens, layouts=layouts)
        return BatchResult(self, batch, r)


def NewDecodingLayerParser(first, *decoders):
    return DecodingLayerParser(first, *decoders)


def _slot(kind):
    """gpk_layout / gpk_fields.present slot of a decoder kind (Payload and Fragment share 7)."""
    return min(kind, _lib.DEC_PAYLOAD) - 1


class BatchResult:
    """Device results of DecodeBatch, with per-packet gopacket views."""

    def __init__(self, parser, batch, r):
        self.parser, self.batch = parser, batch
        self.records, self.err_args, self.flows, self.layouts = r["records"], r["err_args"], r["flows"], \
            r["layouts"]
        self.fields = None  # FIELDS_DTYPE per packet when decoded with fields=True

    def __len__(self):
        return len(self.records)

    def status(self, i):
        return int(self.records[i]["status"])

    def Truncated(self, i):
        return bool(self.status(i) & _lib.ST_TRUNCATED)

    def Decoded(self, i):
        from .engine import decode_codes
        st = self.status(i)
        n = (st >> _lib.ST_NLAYERS_SHIFT) & _lib.ST_NLAYERS_MASK
        if n <= _lib.MAX_INLINE_LAYERS:
            return [LayerType(t) for t in decode_codes(self.records[i]["layers"], n)]
        full = self.parser.ctx().decoded_list_host(self.parser._config(), self.batch.packet(i))
        return [LayerType(t) for t in full]

    def Err(self, i):
        """The error value DecodeLayers returns for packet i (None = nil)."""
        from .engine import format_error
        code = self.status(i) & _lib.ST_ERR_MASK
        if code == 0:
            return None
        a0, a1 = int(self.err_args[2 * i]), int(self.err_args[2 * i + 1])
        if code == 1:
            return UnsupportedLayerType(struct.unpack("<i", struct.pack("<I", a0))[0])
        msg = format_error(code, a0, a1)
        if code in (2, 3, 4) and self.parser.IgnorePanic:
            raise GoPanic(msg[len("panic: "):])
        return GoError(msg)

    def FlowHashes(self, i):
        """(LinkFlow, NetworkFlow, TransportFlow) FastHash values; None where absent."""
        st, n = self.status(i), len(self.records)
        f = self.flows
        return (int(f[i]) if st & _lib.ST_LINK_FLOW else None,
                int(f[n + i]) if st & _lib.ST_NET_FLOW else None,
                int(f[2 * n + i]) if st & _lib.ST_TRANSPORT_FLOW else None)

    def IPv4Checksum(self, i):
        st = self.status(i)
        if not st & _lib.ST_IP4_CSUM:
            return None
        return bool(st & _lib.ST_IP4_VALID), int(self.records[i]["ip4_csum"])

    def L4Checksum(self, i):
        st = self.status(i)
        if not st & _lib.ST_L4_CSUM:
            return None
        return bool(st & _lib.ST_L4_VALID), int(self.records[i]["l4_csum"])

    def IPv4Options(self, i):
        """(Options, Padding) of packet i's IPv4 layer from the device's option
        map (fields=True results): no DecodeFromBytes on the host. None when
        the packet has no IPv4 layer."""
        from .layers import IPv4OptionsFromMap
        f = self._fields_of(i)
        if not int(f["present"]) & (1 << (_lib.DEC_IPV4 - 1)):
            return None
        pkt, s = self._start_of(i, f, _lib.DEC_IPV4, "ip4_start")
        return IPv4OptionsFromMap(pkt, s, int(f["ip4_ihl"]) * 4, f["ip4_opt_map"])

    def TCPOptions(self, i):
        """(Options, Padding, Multipath) of packet i's TCP layer from the
        device's option map (fields=True results). None without a TCP layer."""
        from .layers import TCPOptionsFromMap
        f = self._fields_of(i)
        if not int(f["present"]) & (1 << (_lib.DEC_TCP - 1)):
            return None
        pkt, s = self._start_of(i, f, _lib.DEC_TCP, "tcp_start")
        return TCPOptionsFromMap(pkt, s, int(f["tcp_data_offset"]) * 4, f["tcp_opt_map"])

    def _fields_of(self, i):
        if self.fields is None:
            raise ValueError("option maps need fields=True results")
        return self.fields[i]

    def _start_of(self, i, f, kind, name):
        """(packet bytes, start of the decoder's header): the record's start,
        or, for a header at byte 255 or later (0xFF), the start of its slice
        derived from the decoded list (as Hydrate derives it)."""
        pkt = self.batch.packet(i)
        s = int(f[name])
        if s == 0xFF:
            sl = self._slices(pkt, self.Decoded(i), f) or self._slices_host(pkt, self.Decoded(i))
            s = sl[kind][0]
        return pkt, s

    def Hydrate(self, i, decoded):
        """Make the parser's layer structs and `decoded` look exactly as after
        DecodeLayers(packet i, decoded); returns its error value.

        From layouts=True results each struct is read from its decoder's
        slice. From fields=True results without layouts (the one-launch
        gpk_decode_batch_fields) each struct is filled from the packet's
        gpk_fields record (layers.*._fill), at slices derived from the decoded
        list (_slices); only what the record cannot describe (a stacked IPv4,
        IPv6, Ethernet or UDP, a HopByHop header longer than its option map)
        is read from the packet bytes (counted in host_decodes)."""
        p = self.parser
        if p.first.__int__() not in [int(t) for d in p._decoders.values() for t in d.CanDecode()]:
            # LayersDecoder (layers_decoder.go:12-16): decoded is not truncated
            p.Truncated = False
            return None if p.IgnoreUnsupported else UnsupportedLayerType(p.first)
        decoded[:] = self.Decoded(i)
        p.Truncated = self.Truncated(i)
        err = self.Err(i)
        pkt = self.batch.packet(i)
        if self.layouts is not None:
            lay = self.layouts[i]
            for slot, kind in enumerate(_lib.LAYOUT_SLOTS):
                s = int(lay["start"][slot])
                if s == _lib.LAYOUT_ABSENT:
                    continue
                e = int(lay["end"][slot])
                if slot == 7:
                    kind = _lib.DEC_PAYLOAD if _lib.DEC_PAYLOAD in p._decoders and \
                        LayerTypePayload in decoded else _lib.DEC_FRAGMENT
                inst = p._decoders.get(kind)
                if inst is None:
                    continue
                inst._hydrate(pkt[s:e])
                self._attach(i, kind, inst)
        elif self.fields is not None:
            f = self.fields[i]
            sl = self._slices(pkt, decoded, f)
            fill = True
            if sl is None:  # the record does not describe this stack: read the slices' headers
                self.host_decodes += 1
                sl, fill = self._slices_host(pkt, decoded), False
            pres = int(f["present"])
            for kind, (s, e) in sl.items():
                if not pres >> (_slot(kind)) & 1:
                    continue  # a later DecodeFromBytes of this instance failed: not in the layout either
                if fill:
                    p._decoders[kind]._fill(pkt, s, e, f)
                else:
                    p._decoders[kind]._hydrate(pkt[s:e])
                self._attach(i, kind, p._decoders[kind])
        else:
            raise ValueError("Hydrate needs layouts=True or fields=True results")
        return err

    host_decodes = 0  # packets Hydrate read headers for on the host (fields=True results only)

    def _attach(self, i, kind, inst):
        """The device's flow hash and checksum results on the hydrated struct."""
        st = self.status(i)
        if kind == _lib.DEC_ETHERNET and st & _lib.ST_LINK_FLOW:
            inst._link_hash = int(self.flows[i])
        if kind == _lib.DEC_IPV4 and st & _lib.ST_IP4_CSUM:
            inst._csum = (None, ChecksumVerificationResult(bool(st & _lib.ST_IP4_VALID),
                                                           int(self.records[i]["ip4_csum"]), inst.Checksum))
        if kind in (_lib.DEC_TCP, _lib.DEC_UDP) and st & _lib.ST_L4_CSUM:
            inst._csum = (None, ChecksumVerificationResult(bool(st & _lib.ST_L4_VALID),
                                                           int(self.records[i]["l4_csum"]), inst.Checksum))

    def _kinds(self, decoded):
        """The decoder kind of each decoded LayerType (the parser's container:
        one instance per type, parser.go:74-169)."""
        by_type = {int(t): k for k, d in self.parser._decoders.items() for t in d.CanDecode()}
        return [by_type[int(t)] for t in decoded]

    def _slices(self, pkt, decoded, f):
        """{kind: (start, end)} of the slice each decoder's LAST DecodeFromBytes
        was handed (what gpk_layout records), derived from the decoded list:
        the first decoder gets the whole packet, each next one its
        predecessor's Payload, whose start and end follow from the
        predecessor's fields in the record (layers.payload_end,
        layers.ipv6_payload_start). None when the record cannot give them: a
        decoder whose header length or trim depends on its own fields appears
        twice (the record holds the last instance only), or an inline
        HopByHop is longer than the record's option map."""
        from . import layers as L
        kinds = self._kinds(decoded)
        pres = int(f["present"])
        for k in kinds:
            if not pres >> _slot(k) & 1:  # decoded, then a later instance failed: its fields are gone
                return None
        for k in (_lib.DEC_ETHERNET, _lib.DEC_IPV4, _lib.DEC_IPV6, _lib.DEC_TCP, _lib.DEC_UDP):
            if kinds.count(k) > 1:
                return None
        out, s, e = {}, 0, len(pkt)
        for k in kinds:
            out[k] = (s, e)
            if k == _lib.DEC_ETHERNET:
                s, e = s + 14, L.payload_end(k, pkt, s, e, f)
            elif k == _lib.DEC_DOT1Q:
                s = s + 4
            elif k == _lib.DEC_IPV4:
                s, e = s + int(f["ip4_ihl"]) * 4, L.payload_end(k, pkt, s, e, f)
            elif k == _lib.DEC_IPV6:
                if int(f["ip6_next_header"]) == L.IPProtocolIPv6HopByHop and not L.hbh_map_covers(pkt, s + 40):
                    return None
                s, e = L.ipv6_payload_start(pkt, s, f), L.payload_end(k, pkt, s, e, f)
            elif k == _lib.DEC_IPV6_EXT:
                s = s + pkt[s + 1] * 8 + 8
            elif k == _lib.DEC_TCP:
                s = s + int(f["tcp_data_offset"]) * 4
            elif k == _lib.DEC_UDP:
                s, e = s + 8, L.payload_end(k, pkt, s, e, f)
        # the record's own view of the same decode: presence and the starts it keeps
        got = 0
        for k in out:
            got |= 1 << _slot(k)
        if got != pres:
            raise RuntimeError("fields record presence %#x disagrees with the decoded list (%#x)" % (pres, got))
        for k, name in ((_lib.DEC_IPV4, "ip4_start"), (_lib.DEC_TCP, "tcp_start")):
            if k in out and out[k][0] < 0xFF and out[k][0] != int(f[name]):
                raise RuntimeError("fields record %s %d disagrees with the decoded list (%d)"
                                   % (name, int(f[name]), out[k][0]))
        return out

    def _slices_host(self, pkt, decoded):
        """The same slices, each predecessor's Payload read from its header
        bytes on the host (layers.*._hydrate); the fallback of _slices."""
        out, s, e = {}, 0, len(pkt)
        scratch = {}
        for k in self._kinds(decoded):
            out[k] = (s, e)
            inst = scratch.setdefault(k, type(self.parser._decoders[k])())
            inst._hydrate(pkt[s:e])
            s = s + inst._poff
            e = s + len(inst.LayerPayload())
        return out
