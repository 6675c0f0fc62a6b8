"""pcapgo-shaped capture readers over the native batch indexer (include/gpk_capture.h).

Mirrors the reference's pcapgo package for the ingest side of the path
(SURVEY.md §8(f)1):

  NewNgReader(r, NgReaderOptions) -> NgReader     pcapgo/ngread.go:64-107
  NewReader(r) -> Reader                          pcapgo/read.go:65-71
  reader.ReadPacketData() -> (data, CaptureInfo)  ngread.go:629-632, read.go:122-137
  reader.ReadPacketDataWithOptions()              ngread.go:636-664 (NgPacketOptions)
  reader.LinkType(), SectionInfo(), Interface(i), NInterfaces(), Name(i),
  NNames(), Resolution(), SkipSection()           ngread.go:720-761, 330-335
  NgReaderOptions.SectionEndCallback / StatisticsCallback   ngread.go:32-36
  Reader.Snaplen(), SetSnaplen(), Resolution()    read.go:185-231
  reader.ReadBatch(max) -> PacketBatch            the batch form: packets indexed in
                                                  place in one staging buffer, ready
                                                  for DecodingLayerParser.DecodeBatch

Every record is walked by libgpk's C++ indexer; errors are raised as
PcapgoError carrying the reference's error text (io.EOF is "EOF", raised as
EOFError subclass so `except EOFError` reads like Go's `err == io.EOF`).
Gzip input is inflated transparently, as pcapgo does.
"""
import ctypes
import io
import ipaddress
import struct
import zlib
from dataclasses import dataclass, field

import numpy as np

from . import _lib

LinkTypeNull, LinkTypeEthernet = 0, 1


class PcapgoError(Exception):
    def __init__(self, text, panic=False):
        super().__init__(text)
        self.text = text
        self.panic = panic


class EOFErrorGo(PcapgoError, EOFError):
    """io.EOF"""


def _err(text, panic=False):
    return EOFErrorGo(text) if text == "EOF" else PcapgoError(text, panic)


@dataclass
class NgReaderOptions:  # ngread.go:23-37
    WantMixedLinkType: bool = False
    ErrorOnMismatchingLinkType: bool = False
    SkipUnknownVersion: bool = False
    # SectionEndCallback(interfaces, sectionInfo) at the end of every section but
    # the last (ngread.go:239-245); StatisticsCallback(ifaceID, stats) after every
    # interface statistics block (:485-487). Both are made inside the read call
    # that met the block, before it returns, as the reference makes them.
    SectionEndCallback: object = None
    StatisticsCallback: object = None

    def flags(self):
        return ((_lib.NG_WANT_MIXED_LINKTYPE if self.WantMixedLinkType else 0)
                | (_lib.NG_ERROR_ON_MISMATCHING_LINKTYPE if self.ErrorOnMismatchingLinkType else 0)
                | (_lib.NG_SKIP_UNKNOWN_VERSION if self.SkipUnknownVersion else 0))


DefaultNgReaderOptions = NgReaderOptions()


@dataclass
class CaptureInfo:  # gopacket.CaptureInfo (packet.go)
    Timestamp: tuple  # (unix seconds, nanoseconds) of time.Unix(..).UTC()
    CaptureLength: int
    Length: int
    InterfaceIndex: int = 0
    AncillaryData: list = field(default_factory=list)


@dataclass
class TimestampResolution:  # gopacket.TimestampResolution (time.go)
    Base: int = 0
    Exponent: int = 0


TimestampResolutionMicrosecond = TimestampResolution(10, -6)
TimestampResolutionNanosecond = TimestampResolution(10, -9)


@dataclass
class NgInterfaceStatistics:
    LastUpdate: tuple
    StartTime: tuple
    EndTime: tuple
    Comment: bytes
    PacketsReceived: int
    PacketsDropped: int


@dataclass
class NgInterface:  # pcapgo/pcapng.go
    Name: bytes
    Comment: bytes
    Description: bytes
    Filter: bytes
    OS: bytes
    LinkType: int
    TimestampResolution: int
    TimestampOffset: int
    SnapLength: int
    Statistics: NgInterfaceStatistics

    def Resolution(self):  # NgResolution.ToTimestampResolution (pcapng.go:240-261)
        r = self.TimestampResolution
        return TimestampResolution(2 if r & 0x80 else 10, -(r & 0x7F))


@dataclass
class NgSectionInfo:
    Hardware: bytes
    OS: bytes
    Application: bytes
    Comment: bytes


# NgPacketOptions and its parts (pcapng.go:118-218, 332-350)
NgEpbFlagDirectionMask, NgEpbFlagReceptionTypeMask, NgEpbFlagFCSLengthMask = 0b11, 0b11100, 0b1111100000
NgEpbFlagLinkLayerDependentErrorMask = 0xFFFF0000


@dataclass
class NgEpbFlags:
    Direction: int = 0
    Reception: int = 0
    FCSLen: int = 0
    LinkLayerErr: int = 0

    @classmethod
    def FromUint32(cls, v):  # pcapng.go:174-179
        return cls(v & NgEpbFlagDirectionMask, v & NgEpbFlagReceptionTypeMask, v & NgEpbFlagFCSLengthMask,
                   v & NgEpbFlagLinkLayerDependentErrorMask)


@dataclass
class NgEpbHash:
    Algorithm: int
    Hash: bytes


@dataclass
class NgEpbVerdict:
    Type: int
    Data: bytes


@dataclass
class NgPacketOptions:
    Comments: list = field(default_factory=list)
    Flags: object = None      # NgEpbFlags or None
    Hashes: list = field(default_factory=list)
    DropCount: object = None  # int or None
    PacketID: object = None
    Queue: object = None
    Verdicts: list = field(default_factory=list)


def _packet_options(tlv):
    """readPacketOptions (ngread.go:582-625) over the options the reader kept
    (gpk_capreader_packet_options): the values are read little-endian whatever
    the section's byte order, as the reference reads them."""
    o, p = NgPacketOptions(), 0
    while p + 8 <= len(tlv):
        code, n = struct.unpack_from("<H2xI", tlv, p)
        v = bytes(tlv[p + 8:p + 8 + n])
        p += 8 + ((n + 3) & ~3)
        if code == 1:
            o.Comments.append(v)
        elif code == 2:
            o.Flags = NgEpbFlags.FromUint32(struct.unpack_from("<I", v)[0])
        elif code == 3:
            o.Hashes.append(NgEpbHash(v[0], v[1:]))
        elif code == 4:
            o.DropCount = struct.unpack_from("<Q", v)[0]
        elif code == 5:
            o.PacketID = struct.unpack_from("<Q", v)[0]
        elif code == 6:
            o.Queue = struct.unpack_from("<I", v)[0]
        elif code == 7:
            o.Verdicts.append(NgEpbVerdict(v[0], v[1:]))
    return o


@dataclass
class NgIPAddress:  # pcapng.go:425-431
    Addr: object  # ipaddress.IPv4Address / IPv6Address (netip.AddrFromSlice of 4 / 16 bytes)

    def Len(self):
        return self.Addr.max_prefixlen // 8


@dataclass
class NgEUIAddress:  # pcapng.go:433-439
    Addr: bytes  # the 24 bytes newHWAddress clones (ngread_nrb.go:56-61)

    def Len(self):
        return len(self.Addr)


@dataclass
class NgNameRecord:  # pcapng.go:441-444
    Addr: object
    Names: list


@dataclass
class PacketBatch:
    """Packets indexed in place: packet i is data[offsets[i]:offsets[i]+caplens[i]]."""
    data: np.ndarray      # uint8 staging buffer (the capture stream bytes)
    offsets: np.ndarray   # uint64
    caplens: np.ndarray   # uint32
    ci: np.ndarray        # _lib.CAPINFO_DTYPE

    def __len__(self):
        return len(self.offsets)


def _inflate(raw):
    """Best-effort multistream gunzip: everything that inflates is the stream;
    a truncated or corrupt body ends it there."""
    out, rest = bytearray(), raw
    while rest:
        d = zlib.decompressobj(16 + zlib.MAX_WBITS)
        try:
            out += d.decompress(rest)
        except zlib.error:
            break
        rest = d.unused_data
        if not d.eof or len(rest) < 10 or rest[:2] != b"\x1f\x8b":
            break
    return bytes(out)


class _Source:
    """The capture stream from a bytes object or a binary file object; gzip
    input is inflated first (read.go:80-86, ngread.go:75-91)."""

    def __init__(self, src, chunk=1 << 22):
        self.f = io.BytesIO(bytes(src)) if isinstance(src, (bytes, bytearray, memoryview)) else src
        self.chunk = chunk
        head = self.f.read(2)
        if len(head) == 2 and head == b"\x1f\x8b":
            raw = head + self.f.read()
            if len(raw) < 10:  # gzip.NewReader: the header read hits EOF
                raise _err("unexpected EOF")
            self.f = io.BytesIO(_inflate(raw))
            head = b""
        self.pending = head

    def read(self):
        """Next piece of the (inflated) stream, b"" at the end."""
        if self.pending:
            out, self.pending = self.pending, b""
            return out
        return self.f.read(self.chunk)


class _Indexer:
    def __init__(self, fmt, flags, src):
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(L.gpk_capreader_create(ctypes.byref(h), fmt, flags))
        self.h = h
        self.L = L
        self.src = src
        self.buf = b""   # stream bytes from self.pos on are unconsumed
        self.pos = 0
        self.eof = False

    def __del__(self):
        if getattr(self, "h", None):
            self.L.gpk_capreader_destroy(self.h)
            self.h = None

    def _fill(self):
        piece = self.src.read()
        if not piece:
            self.eof = True
        else:
            self.buf = self.buf[self.pos:] + piece
            self.pos = 0

    def index(self, max_pkts, on_call=None):
        """gpk_capreader_index until max_pkts packets or the reader's end:
        [(data view, offsets, caplens, ci)] per call, and the error (None if
        max_pkts were read). on_call(piece) runs after every call that returned
        packets, while the reader's per-call state (kept options) is valid."""
        L = self.L
        outs, total = [], 0
        while True:
            if self.pos >= len(self.buf) and not self.eof:
                self._fill()
            m = max_pkts - total
            data = np.frombuffer(self.buf, dtype=np.uint8, offset=self.pos) if self.pos < len(self.buf) \
                else np.zeros(0, np.uint8)
            off = np.empty(max(m, 1), np.uint64)
            cap = np.empty(max(m, 1), np.uint32)
            ci = np.empty(max(m, 1), _lib.CAPINFO_DTYPE)
            n, used = ctypes.c_uint64(), ctypes.c_uint64()
            rc = L.gpk_capreader_index(self.h, data.ctypes.data if len(data) else None, len(data), int(self.eof),
                                       off.ctypes.data, cap.ctypes.data, ci.ctypes.data, m, ctypes.byref(n),
                                       ctypes.byref(used))
            if rc < 0:
                _lib.check(rc)
            k = n.value
            if k:
                piece = (data, off[:k], cap[:k], ci[:k])
                outs.append(piece)
                if on_call is not None:
                    on_call(piece)
                total += k
            self.pos += used.value
            if rc == _lib.CAP_END:
                return outs, self.error()
            if rc == _lib.CAP_FULL:
                return outs, None
            if self.eof:  # cannot happen: at the end of the stream every call ends
                return outs, PcapgoError("internal: MORE at end of stream")
            self._fill()

    @staticmethod
    def join(outs):
        """One PacketBatch (its own copy of the packets' bytes, 16 bytes of slack after)."""
        if not outs:
            return PacketBatch(np.zeros(16, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
                               np.zeros(0, _lib.CAPINFO_DTYPE))
        if len(outs) == 1:
            d, o, c, ci = outs[0]
            return PacketBatch(np.concatenate([d, np.zeros(16, np.uint8)]), o, c, ci)
        total = sum(int(c.sum()) for _, _, c, _ in outs)
        data = np.zeros(total + 16, np.uint8)
        offs, pos = [], 0
        for d, o, c, _ in outs:
            for a, ln in zip(o.tolist(), c.tolist()):
                data[pos:pos + ln] = d[a:a + ln]
                offs.append(pos)
                pos += ln
        return PacketBatch(data, np.array(offs, np.uint64), np.concatenate([c for _, _, c, _ in outs]),
                           np.concatenate([ci for _, _, _, ci in outs]))

    def error(self):
        buf = ctypes.create_string_buffer(512)
        eof, panic = ctypes.c_int(), ctypes.c_int()
        n = self.L.gpk_capreader_error(self.h, buf, 512, ctypes.byref(eof), ctypes.byref(panic))
        return _err(buf.raw[:n].decode("latin-1"), bool(panic.value))


class _ReaderBase:
    """Every read is exactly the reference's call: ReadPacketData reads one
    record (so SectionInfo, Interface, Name, SetSnaplen and SkipSection act
    between packets as they do in Go); ReadBatch reads max_pkts of them in one
    native call."""

    def __init__(self, fmt, flags, src):
        self._ix = _Indexer(fmt, flags, _Source(src))
        self._qerr = None
        _, err = self._ix.index(0)  # NewReader / NewNgReader read the header (and first interface) now
        self._events()
        if err is not None:
            raise err

    def _events(self):  # callbacks of what the last call read (NgReader)
        pass

    def _read(self, m, on_call=None):
        if self._qerr is not None:
            e, self._qerr = self._qerr, None
            raise e
        outs, err = self._ix.index(m, on_call)
        self._events()
        if not outs:
            raise err
        self._qerr = err  # raised by the next read, as the next ReadPacketData would return it
        return outs

    def ReadBatch(self, max_pkts=1 << 20):
        """Up to max_pkts packets as one PacketBatch (the packets the next
        ReadPacketData calls would return); raises the terminating error
        (EOFErrorGo at a clean end) once no packet precedes it."""
        return self._ix.join(self._read(max_pkts))

    def _one(self, on_call=None):
        d, o, c, ci = self._read(1, on_call)[0]
        off, cl, r = int(o[0]), int(c[0]), ci[0]
        anc = [int(r["link_type"])] if int(r["link_type"]) >= 0 else []
        return bytes(d[off:off + cl]), CaptureInfo((int(r["ts_sec"]), int(r["ts_nsec"])), cl, int(r["length"]),
                                                   int(r["iface"]), anc)

    def ReadPacketData(self):
        """(data bytes, CaptureInfo), or raises PcapgoError (EOFErrorGo for io.EOF)."""
        return self._one()

    ZeroCopyReadPacketData = ReadPacketData

    def LinkType(self):
        return self._ix.L.gpk_capreader_link_type(self._ix.h)


class Reader(_ReaderBase):
    def __init__(self, r):
        super().__init__(_lib.CAP_PCAP, 0, r)

    def _hdr(self):
        s, mj, mn, ns = ctypes.c_uint32(), ctypes.c_uint16(), ctypes.c_uint16(), ctypes.c_int()
        _lib.check(self._ix.L.gpk_capreader_pcap_header(self._ix.h, ctypes.byref(s), ctypes.byref(mj),
                                                        ctypes.byref(mn), ctypes.byref(ns)))
        return s.value, mj.value, mn.value, bool(ns.value)

    def Snaplen(self):
        return self._hdr()[0]

    def SetSnaplen(self, n):  # read.go:216-218
        _lib.check(self._ix.L.gpk_capreader_set_snaplen(self._ix.h, int(n) & 0xFFFFFFFF))

    def Resolution(self):  # read.go:226-231
        return TimestampResolutionNanosecond if self._hdr()[3] else TimestampResolutionMicrosecond


class NgReader(_ReaderBase):
    def __init__(self, r, options=DefaultNgReaderOptions):
        self._opts = options
        self._fired = 0      # StatisticsCallback / SectionEndCallback calls made so far
        self._fired_sec = 0
        self._fired_stat = 0
        super().__init__(_lib.CAP_PCAPNG, options.flags(), r)

    def _str(self, fn, *args):
        n = fn(self._ix.h, *args, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        fn(self._ix.h, *args, buf, n + 1)
        return buf.raw[:n]

    def _section(self, s):
        f = self._ix.L.gpk_capreader_section_info
        return NgSectionInfo(Hardware=self._str(f, s, 1), OS=self._str(f, s, 2), Application=self._str(f, s, 3),
                             Comment=self._str(f, s, 0))

    @staticmethod
    def _stats(x, comment):
        return NgInterfaceStatistics((x.last_update_sec, x.last_update_nsec), (x.start_time_sec, x.start_time_nsec),
                                     (x.end_time_sec, x.end_time_nsec), comment, x.packets_received,
                                     x.packets_dropped)

    def _iface(self, s, i):
        L = self._ix.L
        x = _lib.NgInterface()
        _lib.check(L.gpk_capreader_interface(self._ix.h, s, i, ctypes.byref(x)))
        f = L.gpk_capreader_interface_str
        return NgInterface(Name=self._str(f, s, i, 0), Comment=self._str(f, s, i, 1),
                           Description=self._str(f, s, i, 2), Filter=self._str(f, s, i, 3), OS=self._str(f, s, i, 4),
                           LinkType=x.link_type, TimestampResolution=x.ts_resolution, TimestampOffset=x.ts_offset,
                           SnapLength=x.snap_length, Statistics=self._stats(x, self._str(f, s, i, 5)))

    def _stat_event(self, k):
        L = self._ix.L
        at, iface, x = ctypes.c_uint64(), ctypes.c_int(), _lib.NgInterface()
        n = L.gpk_capreader_stat_event(self._ix.h, k, ctypes.byref(at), None, ctypes.byref(iface), ctypes.byref(x),
                                       None, 0)
        buf = ctypes.create_string_buffer(max(n, 0) + 1)
        _lib.check(min(0, L.gpk_capreader_stat_event(self._ix.h, k, None, None, None, None, buf, n + 1)))
        return iface.value, self._stats(x, buf.raw[:n])

    def _events(self):
        """The callbacks the reference would have made inside the call just
        made, in the order it would have made them."""
        L, h, o = self._ix.L, self._ix.h, self._opts
        evs = []
        nsec, nst = L.gpk_capreader_nsections(h), L.gpk_capreader_nstat_events(h)
        for s in range(self._fired_sec, nsec):
            seq = ctypes.c_uint64()
            _lib.check(L.gpk_capreader_section_end_at(h, s, None, ctypes.byref(seq)))
            evs.append((seq.value, "section", s))
        for k in range(self._fired_stat, nst):
            seq = ctypes.c_uint64()
            _lib.check(min(0, L.gpk_capreader_stat_event(h, k, None, ctypes.byref(seq), None, None, None, 0)))
            evs.append((seq.value, "stats", k))
        self._fired_sec, self._fired_stat = nsec, nst
        for _, kind, i in sorted(evs):
            if kind == "section" and o.SectionEndCallback is not None:
                o.SectionEndCallback([self._iface(i, j) for j in range(L.gpk_capreader_ninterfaces(h, i))],
                                     self._section(i))
            elif kind == "stats" and o.StatisticsCallback is not None:
                o.StatisticsCallback(*self._stat_event(i))

    def ReadPacketDataWithOptions(self):
        """(data, CaptureInfo, NgPacketOptions) (ngread.go:636-664)."""
        L, got = self._ix.L, []

        def keep(piece):  # the options of the packet this call returned, while the reader still holds them
            tlv, nb = ctypes.c_void_p(), ctypes.c_uint64()
            _lib.check(L.gpk_capreader_packet_options(self._ix.h, 0, ctypes.byref(tlv), ctypes.byref(nb)))
            got.append(ctypes.string_at(tlv, nb.value) if nb.value else b"")

        _lib.check(L.gpk_capreader_keep_options(self._ix.h, 1))
        try:
            data, ci = self._one(keep)
        finally:
            L.gpk_capreader_keep_options(self._ix.h, 0)
        return data, ci, _packet_options(got[0])

    ZeroCopyReadPacketDataWithOptions = ReadPacketDataWithOptions

    def SkipSection(self):
        """ngread.go:330-335: skip the rest of the section and read the next section header."""
        if self._qerr is not None:  # the error the last read met is where the reader stands
            e, self._qerr = self._qerr, None
            raise e
        _lib.check(self._ix.L.gpk_capreader_skip_section(self._ix.h))
        _, err = self._ix.index(0)
        self._events()
        if err is not None:
            raise err

    def SectionInfo(self):
        return self._section(self._ix.L.gpk_capreader_nsections(self._ix.h))

    def NInterfaces(self):
        return self._ix.L.gpk_capreader_ninterfaces(self._ix.h, self._ix.L.gpk_capreader_nsections(self._ix.h))

    def Interface(self, i):
        if i < 0 or i >= self.NInterfaces():
            raise PcapgoError("Interface %d invalid. There are only %d interfaces" % (i, self.NInterfaces()))
        return self._iface(self._ix.L.gpk_capreader_nsections(self._ix.h), i)

    def Resolution(self):  # ngread.go:743-748
        if self._opts.WantMixedLinkType:
            return TimestampResolution()
        return self.Interface(0).Resolution()

    def NNames(self):  # ngread.go:759-761
        return self._ix.L.gpk_capreader_nnames(self._ix.h)

    def Name(self, i):  # ngread.go:751-756 (its error text says "Interface", as the reference's does)
        L = self._ix.L
        if i < 0 or i >= self.NNames():
            raise PcapgoError("Interface %d invalid. There are only %d interfaces" % (i, self.NNames()))
        kind, alen, nn = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        addr = (ctypes.c_uint8 * 24)()
        need = L.gpk_capreader_name(self._ix.h, i, ctypes.byref(kind), addr, ctypes.byref(alen), ctypes.byref(nn),
                                    None, 0)
        buf = ctypes.create_string_buffer(max(need, 1))
        L.gpk_capreader_name(self._ix.h, i, None, None, None, None, buf, need)
        names = buf.raw[:need].split(b"\x00")[:nn.value]
        a = bytes(addr)[:alen.value]
        return NgNameRecord(NgIPAddress(ipaddress.ip_address(a)) if kind.value in (1, 2) else NgEUIAddress(a), names)

    def SectionEnds(self):
        """What SectionEndCallback received so far: [(NgSectionInfo, [NgInterface])]."""
        L = self._ix.L
        out = []
        for s in range(L.gpk_capreader_nsections(self._ix.h)):
            out.append((self._section(s), [self._iface(s, i) for i in range(L.gpk_capreader_ninterfaces(self._ix.h, s))]))
        return out


def NewNgReader(r, options=DefaultNgReaderOptions):
    return NgReader(r, options)


def NewReader(r):
    return Reader(r)
