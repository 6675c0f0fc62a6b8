"""Pure-Python restatement of gopacket's afpacket ring reader.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of the product's
native ring walker (gopacket_amd/csrc/gpk_afpacket.cpp). The product package
never imports it.

What it restates, as a state machine over a bytearray ring (the Go reader's
fields are the attributes of TPacketOracle):

  afpacket/options.go:149-158   defaultOpts
  afpacket/options.go:160-211   parseOptions / options.check (error texts)
  afpacket/afpacket.go:335-367  ZeroCopyReadPacketData (the retry loop, the
                                "empty block" skip, Stats.Packets)
  afpacket/afpacket.go:316-321  releaseCurrentPacket (clearStatus, offset++)
  afpacket/afpacket.go:462-486  getTPacketHeader (ring position arithmetic)
  afpacket/afpacket.go:488-516  pollForFirstPacket (TP_STATUS_USER check)
  afpacket/header.go:59-137     v1/v2/v3 header layouts (tpacket_hdr, tpacket2_hdr,
                                tpacket_block_desc + tpacket_hdr_v1, tpacket3_hdr,
                                tpacketHdrVarient1, sockaddr_ll after tpAlign(hdr))
  afpacket/header.go:147-155    insertVlanHeader (panics below 12 bytes)
  afpacket/header.go:157-268    get{Status,Time,Data,Length,IfaceIndex,VLAN}, next()
  Go stdlib time.Unix(sec, nsec) normalisation

Where Go would block in poll(2) the oracle stops with WAIT and resumes at the
same point on the next call, as the product does. Releases are immediate
(Go's behaviour); the product's deferred release is checked separately.

Pinning: the header layouts are checked against real kernel-filled rings
captured on the loopback interface (tests/golden/afpacket/, made by
tools/capture_afpacket_fixture.py); Go itself cannot run here, so the walk's
Go-specific behaviour (retry on an empty first packet, VLAN insertion, the
panic on short packets) is pinned by the reference's code only: parity for
those is "unpinned" by any reference-produced vector.
"""
import struct

V1, V2, V3 = 0, 1, 2
STATUS_USER = 1
STATUS_VLAN_VALID = 0x10
ALIGN = 16
PAGE_SIZE = 4096
HDR_SIZE = {V1: 0x20, V2: 0x20, V3: 0x30}

WAIT, PACKET, ERROR = "wait", "packet", "error"


def tp_align(x):
    return (x + ALIGN - 1) & ~(ALIGN - 1)


def go_unix(sec, nsec):  # time.Unix normalisation
    if nsec < 0 or nsec >= 1000000000:
        n = int(nsec / 1000000000)  # Go integer division truncates toward zero
        sec += n
        nsec -= n * 1000000000
        if nsec < 0:
            nsec += 1000000000
            sec -= 1
    return sec, nsec


DEFAULT_OPTS = dict(frame_size=4096, block_size=4096 * 128, num_blocks=128, block_timeout_ns=64_000_000,
                    poll_timeout_ns=-1_000_000, version=-1, add_vlan_header=False)


def check_opts(o):
    """options.check (options.go:197-211): error text or None; sets frames_per_block."""
    if o["block_size"] % PAGE_SIZE != 0:
        return "block size %d must be divisible by page size %d" % (o["block_size"], PAGE_SIZE)
    if o["frame_size"] == 0:
        return "runtime error: integer divide by zero"
    if o["block_size"] % o["frame_size"] != 0:
        return "block size %d must be divisible by frame size %d" % (o["block_size"], o["frame_size"])
    if o["num_blocks"] < 1:
        return "num blocks %d must be >= 1" % o["num_blocks"]
    if o["block_timeout_ns"] < 1_000_000:
        return "block timeout"  # Duration formatting not restated; tests match the prefix
    if o["version"] < -1 or o["version"] > V3:
        return "tpacket version InvalidVersion is invalid"
    o["frames_per_block"] = o["block_size"] // o["frame_size"]
    return None


class TPacketOracle:
    def __init__(self, ring, version, opts):
        self.ring = ring  # bytearray (mutated: releases clear statuses)
        self.version = version
        self.o = dict(DEFAULT_OPTS, **opts)
        err = check_opts(self.o)
        assert err is None, err
        fpb, nb, fs = self.o["frames_per_block"], self.o["num_blocks"], self.o["frame_size"]
        self.hdr_bytes = fs * fpb if version == V3 else fs
        self.nhdr = nb if version == V3 else fpb * nb
        self.offset = 0
        self.current = None  # header index
        self.pkt = 0
        self.used = 0
        self.header_next_needed = False
        self.should_release = False
        self.polling = False
        self.packets = 0
        self.dead = False
        self.side = bytearray()  # VLAN-inserted copies (offsets >= len(ring))

    def u16(self, p):
        return struct.unpack_from("<H", self.ring, p)[0]

    def u32(self, p):
        return struct.unpack_from("<I", self.ring, p)[0]

    def i32(self, p):
        return struct.unpack_from("<i", self.ring, p)[0]

    def in_ring(self, p, n):
        return 0 <= p and p + n <= len(self.ring)

    def status(self, h):
        p = h * self.hdr_bytes
        return self.u32(p + 8) if self.version == V3 else self.u32(p)

    def clear_status(self, h):
        p = h * self.hdr_bytes
        if self.version == V3:
            struct.pack_into("<I", self.ring, p + 8, 0)
        elif self.version == V2:
            struct.pack_into("<I", self.ring, p, 0)
        else:
            struct.pack_into("<Q", self.ring, p, 0)

    def get_header(self):  # getTPacketHeader
        lim = self.o["num_blocks"] if self.version == V3 else self.o["frames_per_block"] * self.o["num_blocks"]
        if self.offset >= lim:
            self.offset = 0
        self.current = self.offset
        pos = self.current * self.hdr_bytes
        if self.version == V3:
            if not self.in_ring(pos, 48):
                raise Fault(pos)
            self.pkt = pos + self.u32(pos + 16)
            self.used = 0
        else:
            self.pkt = pos

    def next(self):
        if self.version != V3:
            return False
        self.used += 1
        if self.used >= self.u32(self.current * self.hdr_bytes + 12):
            return False
        p = self.pkt
        nxt = self.u32(p)
        self.pkt += nxt if nxt != 0 else tp_align(self.u32(p + 12) + self.u16(p + 24))
        return True

    def get_length(self):
        p = self.pkt
        return self.u32(p + 16) if self.version == V3 else (self.u32(p + 4) if self.version == V2 else self.u32(p + 8))

    def read(self):
        """One ZeroCopyReadPacketData: (PACKET, (offset, caplen, ts_sec, ts_nsec, length, iface, vlan)),
        (WAIT, None) or (ERROR, text)."""
        if self.dead:
            return ERROR, self.err
        try:
            return self._read()
        except Fault as f:
            self.dead = True
            self.err = "unexpected fault address (ring offset %d)" % f.args[0]
            return ERROR, self.err
        except GoPanic as p:
            self.dead = True
            self.err = p.args[0]
            return ERROR, self.err

    def _read(self):
        hs = HDR_SIZE[self.version]
        resume = self.polling
        while True:
            if resume or self.current is None or not self.header_next_needed or not self.next():
                if not resume:
                    if self.should_release:
                        self.clear_status(self.current)
                        self.offset += 1
                        self.should_release = False
                    self.get_header()
                resume = False
                if not (self.status(self.current) & STATUS_USER):
                    self.polling = True
                    return WAIT, None
                self.polling = False
                self.should_release = True
                if not self.in_ring(self.pkt, hs):
                    raise Fault(self.pkt)
                if self.get_length() == 0:
                    continue  # "We received an empty block"
            break
        p = self.pkt
        if not self.in_ring(p, hs):
            raise Fault(p)
        vlan = -1
        if self.version == V3:
            snap, mac, sec, nsec, tci = self.u32(p + 12), self.u16(p + 24), self.u32(p + 4), self.u32(p + 8), self.u32(p + 32)
            if self.u32(p + 20) & STATUS_VLAN_VALID:
                vlan = tci & 0xFFF
        elif self.version == V2:
            snap, mac, sec, nsec, tci = self.u32(p + 8), self.u16(p + 12), self.u32(p + 16), self.u32(p + 20), self.u16(p + 24)
        else:
            snap, mac, sec, nsec, tci = self.u32(p + 12), self.u16(p + 16), self.u32(p + 20), self.u32(p + 24) * 1000, 0
        ll = p + tp_align(hs)
        d = p + mac
        if not self.in_ring(d, snap):
            raise Fault(d)
        if not self.in_ring(ll, 8):
            raise Fault(ll)
        if self.version != V1 and tci != 0 and self.o["add_vlan_header"]:
            if snap < 12:
                raise GoPanic("runtime error: slice bounds out of range [:12] with capacity %d" % snap)
            data = bytes(self.ring[d:d + 12]) + bytes([0x81, 0, (tci >> 8) & 0xFF, tci & 0xFF]) + bytes(
                self.ring[d + 12:d + snap])
            off = len(self.ring) + len(self.side)
            self.side += data
            caplen = snap + 4
        else:
            off, caplen = d, snap
        ts_sec, ts_nsec = go_unix(sec, nsec)
        self.packets += 1
        self.header_next_needed = True
        return PACKET, (off, caplen, ts_sec, ts_nsec, self.get_length(), self.i32(ll + 4), vlan)

    def data(self, off, caplen):
        if off >= len(self.ring):
            o = off - len(self.ring)
            return bytes(self.side[o:o + caplen])
        return bytes(self.ring[off:off + caplen])

    def read_until_stop(self, max_pkts=1 << 62):
        out = []
        while len(out) < max_pkts:
            kind, v = self.read()
            if kind != PACKET:
                return out, kind, v
            out.append(v)
        return out, "full", None


class Fault(Exception):
    pass


class GoPanic(Exception):
    pass
