"""Pure-Python restatement of gopacket's pcapgo readers (capture ingest).

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of the product's
native batch indexer (gopacket_amd/csrc/gpk_capture.cpp). The product package
never imports it.

What it restates, line by line, as a byte-stream state machine (a position in
the capture plus the reader's state, exactly what Go's bufio-backed reader
consumes per call, so every quirk of the reference's accounting is kept):

  pcapgo/read.go:65-119     NewReader / readHeader (magic, byte order, ns factor,
                            version, snaplen, link type)
  pcapgo/read.go:122-137    Reader.ReadPacketData (snaplen / length checks)
  pcapgo/read.go:169-177    Reader.readPacketHeader (uint32 usec*factor wraps)
  pcapgo/ngread.go:64-107   NewNgReader (gzip peek, first SHB)
  pcapgo/ngread.go:113-137  readBytes / discard (ErrUnexpectedEOF mapping)
  pcapgo/ngread.go:165-193  readBlock (SHB byte-order magic, u32 length)
  pcapgo/ngread.go:196-234  readOption (the option value buffer is reused and
                            keeps stale bytes; zero-length options keep the
                            previous value)
  pcapgo/ngread.go:238-312  readSectionHeader (version skip, section info)
  pcapgo/ngread.go:315-335  skipSection / SkipSection
  pcapgo/ngread.go:338-373  firstInterface
  pcapgo/ngread.go:376-437  readInterfaceDescriptor (time scale; a resolution
                            exponent >= 64 panics with divide by zero)
  pcapgo/ngread.go:440-443  convertTime (uint64 arithmetic)
  pcapgo/ngread.go:446-489  readInterfaceStatistics
  pcapgo/ngread.go:494-580  readPacketHeader (EPB / SPB / PB, link-type filter)
  pcapgo/ngread.go:582-625  readPacketOptions (EPB option panics; the options read are
                            kept per packet, ReadPacketDataWithOptions's opts)
  pcapgo/ngread.go:636-664  ReadPacketDataWithOptions
  pcapgo/ngread_nrb.go:64-130  readNameResolutionBlock (EUI records count 24
                               address bytes: newHWAddress clones r.buf[:], so
                               the reader's 24-byte scratch buffer is tracked
                               through every read into it); Name(i) / NNames()
  NgReaderOptions.StatisticsCallback / SectionEndCallback (ngread.go:32-36): the
                            calls, with the packets returned before each
  pcapgo/ngread_dsb.go:18-39   readDecryptionSecretsBlock
  time.Unix(sec, nsec).UTC() normalisation (Go stdlib time.Unix)

Gzip input (read.go:80-86, ngread.go:75-91) is inflated before the reader sees
it (zlib's published DEFLATE), as the product's file layer does.

Output of read_all(): list of packets (offset into the inflated stream,
caplen, ts_sec, ts_nsec, length, iface, ancillary link type or None), the
terminating Go error text ("EOF" on a clean end), sections seen.
"""
import struct
import zlib

ZERO_TIME_SEC = -62135596800  # time.Time{}.Unix(): Unix(-62135596800, 0).UTC() == time.Time{}
NO_VALUE64 = 0xFFFFFFFFFFFFFFFF  # NgNoValue64 (pcapng.go)
M64 = (1 << 64) - 1
M32 = (1 << 32) - 1

ERR_EOF = "EOF"
ERR_UNEXPECTED_EOF = "unexpected EOF"
ERR_NG_VERSION = "Unknown pcapng Version in Section Header"           # pcapng.go ErrNgVersionMismatch
ERR_NG_LINKTYPE = "Link type of current interface is different from first one"  # ErrNgLinkTypeMismatch

SHB, IDB, PB, SPB, NRB, ISB, EPB, DSB = 0x0A0D0D0A, 1, 2, 3, 4, 5, 6, 0xA
BYTE_ORDER_MAGIC = 0x1A2B3C4D


class GoError(Exception):
    def __init__(self, text, panic=False):
        super().__init__(text)
        self.text = text
        self.panic = panic


def i64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def go_div(a, b):  # Go integer division truncates toward zero
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def unix_utc(sec, nsec):
    """time.Unix(sec, nsec).UTC() as (sec, nsec) with 0 <= nsec < 1e9."""
    if nsec < 0 or nsec >= 1000000000:
        n = go_div(nsec, 1000000000)
        sec += n
        nsec -= n * 1000000000
        if nsec < 0:
            nsec += 1000000000
            sec -= 1
    return i64(sec), nsec


def inflate_if_gzip(raw):
    """read.go:80-86 / ngread.go:75-91: transparently gunzip. Returns (bytes, error-or-None)."""
    if len(raw) >= 2 and raw[0] == 0x1F and raw[1] == 0x8B:
        if len(raw) < 10:  # gzip.NewReader: the 10-byte header read hits EOF
            return b"", ERR_UNEXPECTED_EOF
        # Best effort: everything that inflates is the stream; a truncated or
        # corrupt body ends it there (Go's gzip-specific error texts for that
        # case are not reproduced: parity unpinned).
        out = bytearray()
        rest = raw
        while rest:  # gzip.Reader is multistream by default
            d = zlib.decompressobj(16 + zlib.MAX_WBITS)
            try:
                out += d.decompress(rest)
            except zlib.error:
                break
            if not d.eof:
                break
            rest = d.unused_data
            if len(rest) < 10 or rest[0] != 0x1F or rest[1] != 0x8B:
                break
        return bytes(out), None
    return raw, None


class _Stream:
    """bufio.Reader over an in-memory capture: only the calls pcapgo makes."""

    def __init__(self, data):
        self.d = data
        self.pos = 0

    def read_into(self, n):
        """NgReader.readBytes (ngread.go:113-126): (bytes, n_read, err)."""
        avail = len(self.d) - self.pos
        k = n if n <= avail else avail
        b = self.d[self.pos:self.pos + k]
        self.pos += k
        return b, k, (None if k == n else ERR_UNEXPECTED_EOF)

    def read_full(self, n):
        """io.ReadFull over the bufio.Reader (read.go)."""
        b, k, err = self.read_into(n)
        if err is not None and k == 0 and n > 0:
            err = ERR_EOF
        return b, err

    def discard(self, n):
        avail = len(self.d) - self.pos
        if n <= avail:
            self.pos += n
            return None
        self.pos = len(self.d)
        return ERR_EOF

    def read_until_nul(self):
        i = self.d.find(b"\x00", self.pos)
        if i < 0:
            b = self.d[self.pos:]
            self.pos = len(self.d)
            return b, ERR_EOF
        b = self.d[self.pos:i + 1]
        self.pos = i + 1
        return b, None


class Packet:
    __slots__ = ("offset", "caplen", "ts_sec", "ts_nsec", "length", "iface", "ancil", "opts")

    def __init__(self, offset, caplen, ts, length, iface, ancil, opts=None):
        self.offset, self.caplen = offset, caplen
        self.ts_sec, self.ts_nsec = ts
        self.length, self.iface, self.ancil = length, iface, ancil
        self.opts = opts or []  # the EPB's options as readPacketOptions read them: [(code, value)]

    def key(self):
        return (self.offset, self.caplen, self.ts_sec, self.ts_nsec, self.length, self.iface, self.ancil)


# ---------------------------------------------------------------------------
# pcap (read.go)
# ---------------------------------------------------------------------------
class Reader:
    MAGIC_NS, MAGIC_NS_BE, MAGIC_US, MAGIC_US_BE = 0xA1B23C4D, 0x4D3CB2A1, 0xA1B2C3D4, 0xD4C3B2A1

    def __init__(self, data):
        """NewReader (read.go:65-71) + readHeader (read.go:73-119). Raises GoError."""
        if len(data) < 2:
            raise GoError(ERR_EOF)  # br.Peek(2)
        data, gerr = inflate_if_gzip(data)
        if gerr:
            raise GoError(gerr)
        self.s = _Stream(data)
        buf, err = self.s.read_full(24)
        if err:
            raise GoError(err)
        magic = struct.unpack_from("<I", buf, 0)[0]
        if magic == self.MAGIC_NS:
            self.bo, self.factor = "<", 1
        elif magic == self.MAGIC_NS_BE:
            self.bo, self.factor = ">", 1
        elif magic == self.MAGIC_US:
            self.bo, self.factor = "<", 1000
        elif magic == self.MAGIC_US_BE:
            self.bo, self.factor = ">", 1000
        else:
            raise GoError("Unknown magic %x" % magic)
        self.major, self.minor = struct.unpack_from(self.bo + "HH", buf, 4)
        if self.major != 2:
            raise GoError("Unknown major version %d" % self.major)
        if self.minor != 4:
            raise GoError("Unknown minor version %d" % self.minor)
        self.snaplen = struct.unpack_from(self.bo + "I", buf, 16)[0]
        self.link_type = struct.unpack_from(self.bo + "I", buf, 20)[0] & 0xFFFF  # layers.LinkType is uint16

    def set_snaplen(self, v):  # SetSnaplen (read.go:216-218)
        self.snaplen = v

    def read_packet(self):
        """ReadPacketData (read.go:122-137): Packet, or raises GoError."""
        hdr, err = self.s.read_full(16)  # readPacketHeader (read.go:169-177)
        if err:
            raise GoError(err)
        sec, usec, caplen, length = struct.unpack(self.bo + "IIII", hdr)
        ts = unix_utc(sec, (usec * self.factor) & M32)  # uint32 multiply wraps
        if caplen > self.snaplen:
            raise GoError("capture length exceeds snap length: %d > %d" % (caplen, self.snaplen))
        if caplen > length:
            raise GoError("capture length exceeds original packet length: %d > %d" % (caplen, length))
        off = self.s.pos
        _, err = self.s.read_full(caplen)
        if err:
            raise GoError(err)
        return Packet(off, caplen, ts, length, 0, None)


# ---------------------------------------------------------------------------
# pcapng (ngread.go)
# ---------------------------------------------------------------------------
class NgInterface:
    def __init__(self):
        self.name = self.comment = self.description = self.filter = self.os = b""
        self.link_type = 0
        self.ts_resolution = 0
        self.ts_offset = 0
        self.snap_length = 0
        self.second_mask = self.scale_up = self.scale_down = 0
        self.stats = None  # dict once an ISB was read

    def as_dict(self):
        d = dict(name=self.name, comment=self.comment, description=self.description, filter=self.filter,
                 os=self.os, link_type=self.link_type, ts_resolution=self.ts_resolution, ts_offset=self.ts_offset,
                 snap_length=self.snap_length)
        st = self.stats or dict(last_update=(ZERO_TIME_SEC, 0), start_time=(ZERO_TIME_SEC, 0),
                                end_time=(ZERO_TIME_SEC, 0), comment=b"", received=0, dropped=0)
        d["stats"] = st
        return d


class NgReader:
    def __init__(self, data, want_mixed=False, error_on_mismatch=False, skip_unknown_version=False):
        """NewNgReader (ngread.go:64-107). Raises GoError."""
        self.want_mixed, self.error_on_mismatch, self.skip_unknown = want_mixed, error_on_mismatch, skip_unknown_version
        if len(data) < 2:  # reader.r.Peek(2)
            raise GoError(ERR_UNEXPECTED_EOF if len(data) > 0 else ERR_EOF)
        data, gerr = inflate_if_gzip(data)
        if gerr:
            raise GoError(gerr)
        self.s = _Stream(data)
        self.be = False
        self.typ = 0
        self.length = 0
        self.opt_back = bytearray(1024)  # currentOption.value = make([]byte, 1024)
        self.opt_len = 1024
        self.opt_code = 0
        self.ifaces = []
        self.section = None
        self.link_type = 0
        self.first_section_found = False
        self.active_section = False
        self.ended_sections = []  # SectionEndCallback(interfaces, sectionInfo)
        self.ci = [0, 0, (0, 0), 0, 0]  # iface, caplen, ts, length, (unused)
        self.ancil = None
        self.buf = bytearray(24)  # NgReader.buf: block / option headers land here; EUI names clone all of it
        self.npk = 0  # packets returned
        self.names = []  # nameRecords: (record type, address bytes, [names])
        self.stat_events = []  # StatisticsCallback calls: (packets before, call number, iface, stats dict)
        self.ended_at = []  # SectionEndCallback calls: (packets before, call number)
        self.ncb = 0  # SectionEndCallback + StatisticsCallback calls so far
        self.cur_opts = []
        self.n_secrets = 0
        self._read_block()
        if self.typ != SHB:
            raise GoError("Unknown magic %x" % self.typ)
        self._read_section_header()

    # -- primitives ------------------------------------------------------
    def _u16(self, b, o=0):
        return struct.unpack_from(">H" if self.be else "<H", b, o)[0]

    def _u32(self, b, o=0):
        return struct.unpack_from(">I" if self.be else "<I", b, o)[0]

    def _u64(self, b, o=0):
        return struct.unpack_from(">Q" if self.be else "<Q", b, o)[0]

    def _read(self, n):
        b, k, err = self.s.read_into(n)
        if err:
            raise GoError(err)
        return b

    def _rbuf(self, n, at=0):
        """readBytes(r.buf[at:at+n]): the bytes (a short read's too) land in NgReader.buf."""
        b, k, err = self.s.read_into(n)
        self.buf[at:at + k] = b
        return b, k, err

    def _read_buf(self, n):
        b, k, err = self._rbuf(n)
        if err:
            raise GoError(err)
        return b

    def _discard(self, n):
        if self.s.discard(n):
            raise GoError(ERR_UNEXPECTED_EOF)
        self.length = (self.length - n) & M32

    def _opt_value(self):
        return bytes(self.opt_back[:self.opt_len])

    def _opt_reslice(self, hi):  # value[:hi] reslices up to cap (stale bytes visible)
        return bytes(self.opt_back[:hi])

    # -- ngread.go:165-193 ---------------------------------------------
    def _read_block(self):
        b, k, err = self._rbuf(8)
        if err:
            raise GoError(ERR_EOF if k == 0 else err)
        self.typ = self._u32(b, 0)
        if self.typ == SHB:
            m, k, err = self._rbuf(4, 8)
            if err:
                raise GoError(err)
            if struct.unpack(">I", m)[0] == BYTE_ORDER_MAGIC:
                self.be = True
            elif struct.unpack("<I", m)[0] == BYTE_ORDER_MAGIC:
                self.be = False
            else:
                raise GoError("Wrong byte order value in Section Header")
            self.length = (self._u32(b, 4) - 12) & M32
            return
        self.length = (self._u32(b, 4) - 8) & M32

    # -- ngread.go:196-234 ---------------------------------------------
    def _read_option(self):
        if self.length == 4:
            self.opt_code = 0
            return
        b = self._read_buf(4)
        self.length = (self.length - 4) & M32
        self.opt_code = self._u16(b, 0)
        olen = self._u16(b, 2)
        if self.opt_code == 0:
            if olen != 0:
                raise GoError("End of Options must be zero length")
            return
        if olen != 0:
            if olen < len(self.opt_back):
                self.opt_len = olen
            else:
                self.opt_back = bytearray(olen)
                self.opt_len = olen
            v, k, err = self.s.read_into(olen)
            self.opt_back[:k] = v
            if err:
                raise GoError(err)
            pad = olen % 4
            if pad > 0:
                self._discard(4 - pad)
            self.length = (self.length - olen) & M32

    # -- ngread.go:238-312 ---------------------------------------------
    def _read_section_header(self):
        if self.active_section:
            self.ended_sections.append((self.section, [i.as_dict() for i in self.ifaces]))
            self.ended_at.append((self.npk, self.ncb))
            self.ncb += 1
        self.ifaces = []
        self.n_secrets = 0
        self.names = []
        self.active_section = False
        while True:  # RESTART
            b = self._read_buf(12)
            self.length = (self.length - 12) & M32
            vmaj, vmin = self._u16(b, 0), self._u16(b, 2)
            if vmaj != 1 or vmin != 0:
                if not self.skip_unknown:
                    raise GoError(ERR_NG_VERSION)
                self._discard(self.length)
                self._skip_section()
                continue
            break
        sec = dict(comment=b"", hardware=b"", os=b"", application=b"")
        while True:
            self._read_option()
            c = self.opt_code
            if c == 0:
                break
            if c == 1:
                sec["comment"] = self._opt_value()
            elif c == 2:
                sec["hardware"] = self._opt_value()
            elif c == 3:
                sec["os"] = self._opt_value()
            elif c == 4:
                sec["application"] = self._opt_value()
        self._discard(self.length)
        self.active_section = True
        self.section = sec
        if not self.want_mixed:
            self._first_interface()

    def _skip_section(self):
        while True:
            self._read_block()
            if self.typ == SHB:
                return
            self._discard(self.length)

    # -- ngread.go:338-373 ---------------------------------------------
    def _first_interface(self):
        while True:
            self._read_block()
            t = self.typ
            if t == IDB:
                self._read_interface_descriptor()
                if not self.first_section_found:
                    self.link_type = self.ifaces[0].link_type
                    self.first_section_found = True
                elif self.link_type != self.ifaces[0].link_type:
                    if self.error_on_mismatch:
                        raise GoError(ERR_NG_LINKTYPE)
                    continue
                return
            elif t in (PB, EPB, SPB, ISB):
                raise GoError("A section must have an interface before a packet block")
            elif t == DSB:
                self._read_decryption_secrets()
            elif t == NRB:
                self._read_name_resolution()
            self._discard(self.length)

    # -- ngread.go:376-437 ---------------------------------------------
    def _read_interface_descriptor(self):
        b = self._read_buf(8)
        self.length = (self.length - 8) & M32
        it = NgInterface()
        it.link_type = self._u16(b, 0)
        it.snap_length = self._u32(b, 4)
        while True:
            self._read_option()
            c = self.opt_code
            if c == 0:
                break
            if c == 2:
                it.name = self._opt_value()
            elif c == 1:
                it.comment = self._opt_value()
            elif c == 3:
                it.description = self._opt_value()
            elif c == 11:
                it.filter = self._opt_value()[1:]
            elif c == 12:
                it.os = self._opt_value()
            elif c == 14:
                it.ts_offset = self._u64(self._opt_reslice(8))
            elif c == 9:
                it.ts_resolution = self.opt_back[0]
        self._discard(self.length)
        if it.ts_resolution == 0:
            it.ts_resolution = 6
        exp = it.ts_resolution & 0x7F
        if it.ts_resolution & 0x80:
            it.second_mask = (1 << exp) & M64 if exp < 64 else 0
        else:
            m = 1
            for _ in range(exp):
                m = (m * 10) & M64
            it.second_mask = m
        it.scale_down = 1
        it.scale_up = 1
        if it.second_mask < 1000000000:
            if it.second_mask == 0:
                raise GoError("runtime error: integer divide by zero", panic=True)
            it.scale_up = 1000000000 // it.second_mask
        else:
            it.scale_down = it.second_mask // 1000000000
        self.ifaces.append(it)

    def _convert_time(self, idx, ts):
        it = self.ifaces[idx]
        return (i64((ts // it.second_mask + it.ts_offset) & M64),
                i64(((ts % it.second_mask) * it.scale_up & M64) // it.scale_down))

    def _time(self, idx, ts):
        return unix_utc(*self._convert_time(idx, ts))

    # -- ngread.go:446-489 ---------------------------------------------
    def _read_interface_statistics(self):
        b = self._read_buf(12)
        self.length = (self.length - 12) & M32
        idx = self._u32(b, 0)
        ts = (self._u32(b, 4) << 32) | self._u32(b, 8)
        if idx >= len(self.ifaces):
            raise GoError("Interface id %d not present in section (have only %d interfaces)" % (idx, len(self.ifaces)))
        st = dict(last_update=(ZERO_TIME_SEC, 0), start_time=(ZERO_TIME_SEC, 0), end_time=(ZERO_TIME_SEC, 0),
                  comment=b"", received=NO_VALUE64, dropped=NO_VALUE64)
        self.ifaces[idx].stats = st
        st["last_update"] = self._time(idx, ts)
        while True:
            self._read_option()
            c = self.opt_code
            if c == 0:
                break
            if c == 1:
                st["comment"] = self._opt_value()
            elif c in (2, 3):
                v = self._opt_reslice(8)
                t = (self._u32(v, 0) << 32) | self._u32(v, 4)
                st["start_time" if c == 2 else "end_time"] = self._time(idx, t)
            elif c == 4:
                st["received"] = self._u64(self._opt_reslice(8))
            elif c == 5:
                st["dropped"] = self._u64(self._opt_reslice(8))
        self._discard(self.length)
        self.stat_events.append((self.npk, self.ncb, idx, dict(st)))  # StatisticsCallback(ifaceID, *stats)
        self.ncb += 1

    # -- ngread_dsb.go:18-39 --------------------------------------------
    def _read_decryption_secrets(self):
        b, k, err = self._rbuf(8)
        if err:
            raise GoError("could not read DecryptionSecret Header block length: %s" % err)
        self.length = (self.length - 8) & M32
        slen = self._u32(b, 4)
        _, k, err = self.s.read_into(slen)
        if err:
            raise GoError("could not read %d bytes from DecryptionSecret payload: %s" % (slen, err))
        self.length = (self.length - slen) & M32
        self.n_secrets += 1

    # -- ngread_nrb.go:64-130 -------------------------------------------
    def _read_name_resolution(self):
        while self.length > 0:
            b, k, err = self._rbuf(4)
            if err:
                raise GoError("could not read NameRecord Header block length: %s" % err)
            self.length = (self.length - 4) & M32
            rtype, rlen = self._u16(b, 0), self._u16(b, 2)
            length = min(rlen, self.length)
            padding = (4 - length % 4) if length % 4 else 0
            if rtype in (1, 2):
                _, k, err = self._rbuf(4 if rtype == 1 else 16)
                if err:
                    raise GoError("could not read %s address: could not read IP address: %s"
                                  % ("IPv4" if rtype == 1 else "IPv6", err))
                alen = 4 if rtype == 1 else 16
                addr = bytes(self.buf[:alen])  # netip.AddrFromSlice(r.buf[:length])
            elif rtype in (3, 4):
                _, k, err = self._rbuf(6 if rtype == 3 else 8)
                if err:
                    raise GoError("could not read %s address: could not read EUI address: %s"
                                  % ("EUI-48" if rtype == 3 else "EUI-64", err))
                alen = 24  # newHWAddress(r.buf[:]) clones the whole 24-byte buffer
                addr = bytes(self.buf)
            elif rtype == 0:
                break
            else:
                if self.s.discard(length + padding):
                    raise GoError("could not discard unknown name record: %s" % ERR_UNEXPECTED_EOF)
                self.length = (self.length - (length + padding)) & M32
                continue
            self.length = (self.length - length) & M32
            length -= alen
            names = []
            while length > 0:
                bstr, err = self.s.read_until_nul()
                if err:
                    raise GoError("could not read name: %s" % err)
                length -= len(bstr)
                names.append(bytes(bstr).strip(b"\x00"))  # bytes.Trim(bstr, "\x00")
            self.names.append((rtype, addr, names))
            self._discard(padding)
        self._discard(self.length)

    # -- ngread.go:494-580 ---------------------------------------------
    def _read_packet_header(self):
        while True:  # RESTART
            while True:  # FIND_PACKET
                self._read_block()
                t = self.typ
                if t == EPB:
                    b = self._read_buf(20)
                    self.length = (self.length - 20) & M32
                    idx = self._u32(b, 0)
                    if idx >= len(self.ifaces):
                        raise GoError("Interface id %d not present in section (have only %d interfaces)"
                                      % (idx, len(self.ifaces)))
                    ts = self._time(idx, (self._u32(b, 4) << 32) | self._u32(b, 8))
                    self.ci = [idx, self._u32(b, 12), ts, self._u32(b, 16)]
                    break
                elif t == SPB:
                    b = self._read_buf(4)
                    self.length = (self.length - 4) & M32
                    length = self._u32(b, 0)
                    caplen = length
                    if len(self.ifaces) == 0:
                        self.ci = [0, caplen, (ZERO_TIME_SEC, 0), length]
                        raise GoError("At least one Interface is needed for a packet")
                    sl = self.ifaces[0].snap_length
                    if sl != 0 and caplen > sl:
                        caplen = sl
                    self.ci = [0, caplen, (ZERO_TIME_SEC, 0), length]
                    break
                elif t == IDB:
                    self._read_interface_descriptor()
                elif t == ISB:
                    self._read_interface_statistics()
                elif t == SHB:
                    self._read_section_header()
                elif t == PB:
                    b = self._read_buf(20)
                    self.length = (self.length - 20) & M32
                    idx = self._u16(b, 0)
                    if idx >= len(self.ifaces):
                        raise GoError("Interface id %d not present in section (have only %d interfaces)"
                                      % (idx, len(self.ifaces)))
                    ts = self._time(idx, (self._u32(b, 4) << 32) | self._u32(b, 8))
                    self.ci = [idx, self._u32(b, 12), ts, self._u32(b, 16)]
                    break
                elif t == NRB:
                    self._read_name_resolution()
                else:
                    self._discard(self.length)
            if not self.want_mixed:
                if self.ifaces[self.ci[0]].link_type != self.link_type:
                    self._discard(self.length)
                    if self.error_on_mismatch:
                        raise GoError(ERR_NG_LINKTYPE)
                    continue
                self.ancil = None
                return
            self.ancil = self.ifaces[self.ci[0]].link_type
            return

    # -- ngread.go:582-625 ---------------------------------------------
    def _read_packet_options(self):
        while True:
            self._read_option()
            c = self.opt_code
            if c == 0:
                return
            n = self.opt_len
            if c in (2, 6) and n < 4:  # binary.LittleEndian.Uint32: _ = b[3]
                raise GoError("runtime error: index out of range [3] with length %d" % n, panic=True)
            if c in (4, 5) and n < 8:  # binary.LittleEndian.Uint64: _ = b[7]
                raise GoError("runtime error: index out of range [7] with length %d" % n, panic=True)
            self.cur_opts.append((c, self._opt_value()))

    # -- ngread.go:315-335 ---------------------------------------------
    def skip_section(self):
        """SkipSection: skipSection, then readSectionHeader. Raises GoError."""
        self._skip_section()
        self._read_section_header()

    # -- ngread.go:636-664 ---------------------------------------------
    def read_packet(self):
        """ReadPacketDataWithOptions: Packet (opts: the options read), or raises GoError."""
        self.cur_opts = []
        self._read_packet_header()
        idx, caplen, ts, length = self.ci
        off = self.s.pos
        self._read(caplen)
        self.length = (self.length - caplen) & M32
        pad = (4 - (caplen & 3)) & 3
        if pad > 0:
            self._discard(pad)
        if self.typ == EPB:
            self._read_packet_options()
        self._discard(self.length)
        self.npk += 1
        return Packet(off, caplen, ts, length, idx, self.ancil, self.cur_opts)

    def section_state(self):
        return self.section, [i.as_dict() for i in self.ifaces]


def read_all(data, kind="ng", limit=None, **opts):
    """Drain a reader the way a ReadPacketData loop does: stop at the first error.
    Returns dict(packets, err, panic, stream, link_type, sections)."""
    try:
        r = NgReader(data, **opts) if kind == "ng" else Reader(data)
    except GoError as e:
        return dict(packets=[], err=e.text, panic=e.panic, open_err=True, stream=b"", link_type=0, sections=[])
    pk = []
    err, panic = None, False
    while limit is None or len(pk) < limit:
        try:
            pk.append(r.read_packet())
        except GoError as e:
            err, panic = e.text, e.panic
            break
    out = dict(packets=pk, err=err, panic=panic, open_err=False, stream=r.s.d, link_type=r.link_type)
    if kind == "ng":
        out["sections"] = list(r.ended_sections) + [r.section_state()]
    return out
