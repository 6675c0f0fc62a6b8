"""Test helpers: golden vectors, pcap reading, batch packing and a
structure-aware packet fuzzer aimed at the parity traps of SURVEY.md §8
(P1-P12): unknown next types, stacked layers, IPv6 HopByHop/jumbograms,
IPv4/TCP option edge cases, MPTCP options that panic in the reference,
truncation at every boundary.
"""
import json
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def golden():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        return json.load(f)


def golden_bytes(name):
    return bytes.fromhex(golden()[name]["hex"])


def read_pcap(path):
    """Classic pcap (pcapgo/read.go:65-177 semantics for the fixture files)."""
    raw = open(path, "rb").read()
    magic = struct.unpack("<I", raw[:4])[0]
    if magic in (0xa1b2c3d4, 0xa1b23c4d):
        e = "<"
    else:
        e = ">"
    _, _, _, _, _, snaplen, link = struct.unpack(e + "IHHiIII", raw[:24])
    pos, out = 24, []
    while pos + 16 <= len(raw):
        _, _, incl, orig = struct.unpack(e + "IIII", raw[pos:pos + 16])
        pos += 16
        out.append(raw[pos:pos + incl])
        pos += incl
    return link, out


def pack(packets, align=1, pad=0):
    """Packed batch: (data uint8, offsets uint64, caplens uint32). `align`
    places each packet at a multiple of `align` (1 = contiguous)."""
    offs, off = [], pad
    for p in packets:
        off = (off + align - 1) // align * align
        offs.append(off)
        off += len(p)
    data = np.zeros(off + 64, np.uint8)
    for o, p in zip(offs, packets):
        data[o:o + len(p)] = np.frombuffer(p, np.uint8) if len(p) else []
    return data, np.array(offs, np.uint64), np.array([len(p) for p in packets], np.uint32)


def ipv6_udp_jumbogram(checksum=0, hbh16=False):
    """The packet layers/tcpip_test.go:138-186 (TestIPv6JumbogramUDPChecksum)
    serializes, rebuilt from the test's code: IPv6 2001:db8::1 -> 2001:db8::2,
    HopLimit 64, Length 0 (ip6.go:202-208, jumbo); the HopByHop header
    addIPv6JumboOption adds (ip6.go:80-102: NextHeader UDP, HdrExtLen 0, the
    Jumbo TLV 0xC2/4 at offset 2, no padding: serializeIPv6HeaderTLVOptions
    ip6.go:368-408) holding the payload length from the HopByHop header on
    (setIPv6PayloadJumboLength ip6.go:105-134: 8 + 8 + 65536); UDP 12345 ->
    9999 with Length 0 (udp.go:65-81, jumbo) and 65536 bytes of 0xfe.
    hbh16: a jumbogram whose IPv6 Payload is the UDP segment as DecodeLayers
    slices it: a 16-byte HopByHop header (PadN, the Jumbo TLV at 4n+2, PadN)
    whose bytes 4-5 are 0, so the UDP decoder reads them as a jumbo Length 0
    (udp.go:49-50) and sums the whole rest of the packet."""
    src = bytes.fromhex("20010db8000000000000000000000001")
    dst = bytes.fromhex("20010db8000000000000000000000002")
    payload = b"\xfe" * 65536
    hbh = bytes([17, 0, 0xC2, 4]) + struct.pack(">I", 8 + 8 + len(payload))
    if hbh16:
        hbh = bytes([17, 1, 1, 2, 0, 0, 0xC2, 4]) + struct.pack(">I", 16 + 8 + len(payload)) + bytes([1, 2, 0, 0])
    udp = struct.pack(">HHHH", 12345, 9999, 0, checksum)
    ip6 = struct.pack(">IHBB16s16s", 0x60000000, 0, 0, 64, src, dst)
    return ip6 + hbh + udp + payload


# ---------------------------------------------------------------------------
# structure-aware fuzzer

ETHERTYPES = [0x0800, 0x86dd, 0x8100, 0x88a8, 0x0806, 0x6558, 0x0000, 0x0005, 0x05ff, 0x0600, 0xffff, 0x1234,
              0x8847]
PROTOS = [6, 17, 4, 41, 0, 43, 44, 60, 59, 1, 58, 47, 200, 255]


class Fuzzer:
    def __init__(self, seed):
        self.r = np.random.default_rng(seed)

    def u(self, n):
        return int(self.r.integers(0, n))

    def pick(self, xs):
        return xs[self.u(len(xs))]

    def rbytes(self, n):
        return bytes(self.r.integers(0, 256, n, dtype=np.uint8))

    def port(self, udp):
        # mostly payload ports, sometimes ports with application LayerTypes (P1/unsupported)
        if self.u(5) == 0:
            return self.pick([53, 443, 502, 2222, 3868, 44818, 4789, 123, 67, 5060, 6081, 0, 80])
        return 1024 + self.u(60000)

    def tcp_options(self):
        out = b""
        for _ in range(self.u(6)):
            k = self.u(12)
            if k == 0:
                out += b"\x00"
            elif k == 1:
                out += b"\x01"
            elif k == 2:
                out += bytes([2, 4]) + self.rbytes(2)
            elif k == 3:
                out += bytes([8, 10]) + self.rbytes(8)
            elif k == 4:  # bad lengths
                out += bytes([self.u(256), self.pick([0, 1, 2, 3, 40, 255])])
            elif k in (5, 6, 7, 8):  # MPTCP, random subtype/length, often short
                sub = self.u(16)
                ln = self.pick([0, 1, 2, 3, 4, 8, 10, 12, 16, 18, 20, 22, 24, 28, 30, self.u(40)])
                body = bytes([30, ln, (sub << 4) | self.u(16), self.u(256)]) + self.rbytes(self.u(28))
                out += body[:max(2, min(len(body), ln if ln else 3))] if self.u(3) else body[:self.u(len(body) + 1)]
            else:
                out += self.rbytes(self.u(6))
        return out

    def ip4_options(self):
        out = b""
        for _ in range(self.u(4)):
            k = self.u(6)
            if k == 0:
                out += b"\x00"
            elif k == 1:
                out += b"\x01"
            elif k == 2:
                ln = self.pick([0, 1, 2, 3, 4, 11, 40])
                out += bytes([self.pick([7, 68, 130, 136, 148]), ln]) + self.rbytes(max(0, ln - 2))
            else:
                out += self.rbytes(self.u(8))
        return out

    def l4(self, proto, room):
        if proto == 6:
            opts = self.tcp_options() if self.u(3) == 0 else b""
            if self.u(2):
                opts += b"\x00" * ((4 - len(opts) % 4) % 4)
            doff = min(15, 5 + len(opts) // 4) if self.u(8) else self.u(16)
            h = struct.pack(">HHIIBBHHH", self.port(0), self.port(0), self.u(1 << 32), self.u(1 << 32),
                            doff << 4 | self.u(2), self.u(256), self.u(65536), self.u(65536), 0)
            return h + opts + self.rbytes(self.u(max(1, room)))
        if proto == 17:
            body = self.rbytes(self.u(max(1, room)))
            ln = 8 + len(body) if self.u(4) else self.pick([0, 1, 7, 8, 9, 65535, self.u(65536)])
            return struct.pack(">HHHH", self.port(1), self.port(1), ln, self.pick([0, self.u(65536)])) + body
        return self.rbytes(self.u(max(1, room)))

    def ip4(self, depth):
        proto = self.pick(PROTOS) if self.u(3) == 0 else self.pick([6, 17, 6, 17, 4])
        opts = self.ip4_options() if self.u(4) == 0 else b""
        if self.u(2):
            opts += b"\x00" * ((4 - len(opts) % 4) % 4)
        ihl = min(15, 5 + len(opts) // 4) if self.u(10) else self.u(16)
        inner = self.inner(proto, depth)
        total = 20 + len(opts) + len(inner)
        ln = total if self.u(6) else self.pick([0, total - 1, total + 5, 19, 20, self.u(65536)])
        ff = self.pick([0x4000, 0x4000, 0, 0x2000, 0x0001, self.u(65536)]) if self.u(4) == 0 else 0x4000
        h = struct.pack(">BBHHHBBH4s4s", 0x40 | ihl, 0, ln & 0xffff, self.u(65536), ff, 64, proto, self.u(65536),
                        self.rbytes(4), self.rbytes(4))
        return h + opts + inner

    def hbh(self, nh):
        opts = b""
        k = self.u(6)
        if k == 0:
            opts = bytes([0xC2, 4]) + struct.pack(">I", self.pick([0, 65535, 65536, 70000, self.u(1 << 32)]))
        elif k == 1:
            opts = bytes([0xC2, self.pick([2, 3, 5])]) + self.rbytes(5)
        elif k == 2:
            opts = b"\x00" * self.u(6)
        else:
            opts = bytes([1, self.u(6)]) + self.rbytes(6)
        body = bytes([nh, self.pick([0, 0, 1, 2, 255])]) + opts
        pad = (8 - len(body) % 8) % 8
        return body + b"\x00" * pad

    def ip6(self, depth):
        proto = self.pick(PROTOS) if self.u(3) == 0 else self.pick([6, 17, 6, 17, 0, 60])
        ext = b""
        nh = proto
        if proto == 0:
            nh = self.pick([6, 17, 59, 0, 60])
            ext = self.hbh(nh)
        elif proto in (43, 44, 60):
            nh = self.pick([6, 17, 59, 60])
            hl = self.pick([0, 0, 1, 40])
            ext = bytes([nh, hl]) + self.rbytes(6 + 8 * hl)
        inner = self.inner(nh, depth)
        plen = len(ext) + len(inner)
        ln = plen if self.u(5) else self.pick([0, plen - 1, plen + 10, self.u(65536)])
        h = struct.pack(">IHBB16s16s", 0x60000000 | self.u(1 << 20), ln & 0xffff, proto, 64, self.rbytes(16),
                        self.rbytes(16))
        return h + ext + inner

    def inner(self, proto, depth):
        if depth > 3:
            return self.rbytes(self.u(40))
        if proto == 4 and self.u(2):
            return self.ip4(depth + 1)
        if proto == 41 and self.u(2):
            return self.ip6(depth + 1)
        return self.l4(proto, 64 if self.u(4) else 1600)

    def ether(self):
        tags = b""
        for _ in range(self.pick([0, 0, 0, 1, 2, 3])):
            tags += struct.pack(">HH", self.pick([0x8100, 0x88a8]), self.u(65536))
        et = self.pick(ETHERTYPES) if self.u(4) == 0 else self.pick([0x0800, 0x0800, 0x86dd])
        if et == 0x0800:
            body = self.ip4(0)
        elif et == 0x86dd:
            body = self.ip6(0)
        elif et < 0x600:
            body = self.rbytes(self.u(80))
        else:
            body = self.rbytes(self.u(100))
        if tags:
            # tags: first tag type goes in the Ethernet header, each tag carries the next type
            types = [struct.unpack(">H", tags[i:i + 2])[0] for i in range(0, len(tags), 4)]
            tci = [tags[i + 2:i + 4] for i in range(0, len(tags), 4)]
            seq = b""
            for k in range(len(types)):
                nxt = types[k + 1] if k + 1 < len(types) else et
                seq += tci[k] + struct.pack(">H", nxt)
            hdr = self.rbytes(12) + struct.pack(">H", types[0]) + seq
        else:
            hdr = self.rbytes(12) + struct.pack(">H", et)
        return hdr + body

    def packet(self):
        p = self.ether()
        k = self.u(10)
        if k == 0:
            p = p[:self.u(len(p) + 1)]  # truncate anywhere
        elif k == 1:
            b = bytearray(p)
            for _ in range(1 + self.u(4)):
                if b:
                    b[self.u(min(len(b), 96))] = self.u(256)
            p = bytes(b)
        elif k == 2:
            p = p + b"\x00" * self.u(30)  # Ethernet trailer / padding (P10)
        return p


def fuzz_packets(seed, n):
    f = Fuzzer(seed)
    return [f.packet() for _ in range(n)]
