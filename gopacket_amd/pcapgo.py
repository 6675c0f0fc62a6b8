"""pcapgo-shaped capture readers over the native batch indexer (include/gpk_capture.h).

Mirrors the reference's pcapgo package for the ingest side of the path
(SURVEY.md §8(f)1):

  NewNgReader(r, NgReaderOptions) -> NgReader     pcapgo/ngread.go:64-106
  NewReader(r) -> Reader                          pcapgo/read.go:64-70
  reader.ReadPacketData() -> (data, CaptureInfo)  ngread.go:636-640, read.go:124-140
  reader.LinkType(), SectionInfo(), Interface(i), NInterfaces()
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
class NgReaderOptions:  # ngread.go:23-37 (the callbacks are replaced by SectionEnds())
    WantMixedLinkType: bool = False
    ErrorOnMismatchingLinkType: bool = False
    SkipUnknownVersion: bool = False

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


@dataclass
class NgSectionInfo:
    Hardware: bytes
    OS: bytes
    Application: bytes
    Comment: bytes


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
    input is inflated first (read.go:74-84, ngread.go:80-95)."""

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
        self.buf = b""   # unconsumed stream bytes
        self.eof = False
        self.done_err = None

    def __del__(self):
        if getattr(self, "h", None):
            self.L.gpk_capreader_destroy(self.h)
            self.h = None

    def _fill(self):
        piece = self.src.read()
        if not piece:
            self.eof = True
        else:
            self.buf += piece

    def batch(self, max_pkts):
        """Index up to max_pkts packets; returns (PacketBatch, error-or-None)."""
        L = self.L
        outs = []
        total = 0
        while True:
            if not self.buf and not self.eof:
                self._fill()
            data = np.frombuffer(self.buf, dtype=np.uint8) if self.buf else np.zeros(0, np.uint8)
            m = max_pkts - total
            off = np.empty(m, np.uint64)
            cap = np.empty(m, np.uint32)
            ci = np.empty(m, _lib.CAPINFO_DTYPE)
            n, used = ctypes.c_uint64(), ctypes.c_uint64()
            rc = L.gpk_capreader_index(self.h, data.ctypes.data if len(data) else None, len(data), int(self.eof),
                                       off.ctypes.data, cap.ctypes.data, ci.ctypes.data, m, ctypes.byref(n),
                                       ctypes.byref(used))
            if rc < 0:
                _lib.check(rc)
            k = n.value
            if k:  # the staging copy keeps 16 bytes of readable slack after the last packet
                outs.append((np.concatenate([data, np.zeros(16, np.uint8)]), off[:k], cap[:k], ci[:k]))
                total += k
            self.buf = self.buf[used.value:]
            if rc == _lib.CAP_END:
                return self._join(outs), self.error()
            if rc == _lib.CAP_FULL:
                break
            if self.eof:  # cannot happen: at the end of the stream every call ends
                return self._join(outs), PcapgoError("internal: MORE at end of stream")
            self._fill()
        return self._join(outs), None

    @staticmethod
    def _join(outs):
        if not outs:
            return PacketBatch(np.zeros(16, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
                               np.zeros(0, _lib.CAPINFO_DTYPE))
        if len(outs) == 1:
            d, o, c, ci = outs[0]
            return PacketBatch(d, o, c, ci)
        # several chunks: repack their packets into one buffer (16 bytes of slack after)
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
    def __init__(self, fmt, flags, src):
        self._ix = _Indexer(fmt, flags, _Source(src))
        # NewReader / NewNgReader read the header (and first interface) now
        self._queue = None
        self._qerr = None
        b, err = self._ix.batch(0)
        if err is not None:
            raise err

    def _take(self, m):
        if self._qerr is not None:
            e, self._qerr = self._qerr, None
            raise e
        b, err = self._ix.batch(m)
        if len(b) == 0:
            raise err
        self._qerr = err  # raised by the next read, as the next ReadPacketData would return it
        return b

    def ReadBatch(self, max_pkts=1 << 20):
        """Up to max_pkts packets as one PacketBatch (the packets the next
        ReadPacketData calls would return); raises the terminating error
        (EOFErrorGo at a clean end) once no packet precedes it."""
        if self._queue is not None and self._qi < len(self._queue):
            raise PcapgoError("ReadBatch after a partial ReadPacketData batch")
        return self._take(max_pkts)

    def ReadPacketData(self):
        """(data bytes, CaptureInfo), or raises PcapgoError (EOFErrorGo for io.EOF)."""
        if self._queue is None or self._qi >= len(self._queue):
            self._queue, self._qi = None, 0
            self._queue = self._take(256)
        b, i = self._queue, self._qi
        self._qi += 1
        o, c = int(b.offsets[i]), int(b.caplens[i])
        r = b.ci[i]
        anc = [int(r["link_type"])] if int(r["link_type"]) >= 0 else []
        return bytes(b.data[o:o + c]), CaptureInfo((int(r["ts_sec"]), int(r["ts_nsec"])), c, int(r["length"]),
                                                   int(r["iface"]), anc)

    ZeroCopyReadPacketData = ReadPacketData

    def LinkType(self):
        return self._ix.L.gpk_capreader_link_type(self._ix.h)


class Reader(_ReaderBase):
    def __init__(self, r):
        super().__init__(_lib.CAP_PCAP, 0, r)

    def Snaplen(self):
        s = ctypes.c_uint32()
        _lib.check(self._ix.L.gpk_capreader_pcap_header(self._ix.h, ctypes.byref(s), None, None, None))
        return s.value


class NgReader(_ReaderBase):
    def __init__(self, r, options=DefaultNgReaderOptions):
        super().__init__(_lib.CAP_PCAPNG, options.flags(), r)

    def _str(self, fn, *args):
        L = self._ix.L
        n = fn(self._ix.h, *args, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        fn(self._ix.h, *args, buf, n + 1)
        return buf.raw[:n]

    def _section(self, s):
        f = self._ix.L.gpk_capreader_section_info
        return NgSectionInfo(Hardware=self._str(f, s, 1), OS=self._str(f, s, 2), Application=self._str(f, s, 3),
                             Comment=self._str(f, s, 0))

    def _iface(self, s, i):
        L = self._ix.L
        x = _lib.NgInterface()
        _lib.check(L.gpk_capreader_interface(self._ix.h, s, i, ctypes.byref(x)))
        f = L.gpk_capreader_interface_str
        st = NgInterfaceStatistics((x.last_update_sec, x.last_update_nsec), (x.start_time_sec, x.start_time_nsec),
                                   (x.end_time_sec, x.end_time_nsec), self._str(f, s, i, 5), x.packets_received,
                                   x.packets_dropped)
        return NgInterface(Name=self._str(f, s, i, 0), Comment=self._str(f, s, i, 1),
                           Description=self._str(f, s, i, 2), Filter=self._str(f, s, i, 3), OS=self._str(f, s, i, 4),
                           LinkType=x.link_type, TimestampResolution=x.ts_resolution, TimestampOffset=x.ts_offset,
                           SnapLength=x.snap_length, Statistics=st)

    def SectionInfo(self):
        return self._section(self._ix.L.gpk_capreader_nsections(self._ix.h))

    def NInterfaces(self):
        return self._ix.L.gpk_capreader_ninterfaces(self._ix.h, self._ix.L.gpk_capreader_nsections(self._ix.h))

    def Interface(self, i):
        if i < 0 or i >= self.NInterfaces():
            raise PcapgoError("Interface %d invalid. There are only %d interfaces" % (i, self.NInterfaces()))
        return self._iface(self._ix.L.gpk_capreader_nsections(self._ix.h), i)

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
