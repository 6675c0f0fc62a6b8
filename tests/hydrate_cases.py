"""Shared by the Hydrate-from-fields tests (CPU: the oracle's records and
fields; GPU: the device's): IPv6 HopByHop packets of every option shape the
map covers, and a struct-by-struct comparison of two hydration paths."""
import random
import struct

from gopacket_amd import _lib
from gopacket_amd import gopacket as G
from gopacket_amd import layers as L


def hbh_header(rng, nh, hl=None, jumbo=None):
    """An inline HopByHop header: NextHeader nh, HeaderLength hl (0..3), a mix
    of Pad1, PadN, Router Alert and (when jumbo is not None) a Jumbo Payload
    option (ip6.go:327-346, 509-526), padded to (hl + 1) * 8 bytes."""
    hl = rng.choice([0, 0, 1, 2, 3]) if hl is None else hl
    room = hl * 8 + 6
    opts = b""
    if jumbo is not None:
        opts += bytes([0xC2, 4]) + struct.pack(">I", jumbo)
    while len(opts) < room:
        left = room - len(opts)
        k = rng.randrange(4)
        if k == 0 or left < 2:
            opts += b"\x00"  # Pad1
        elif k == 1:
            n = rng.randrange(0, left - 1)
            opts += bytes([1, n]) + bytes(n)  # PadN
        elif k == 2 and left >= 4:
            opts += bytes([5, 2]) + struct.pack(">H", rng.randrange(65536))  # Router Alert
        else:
            opts += b"\x00"
    return bytes([nh, hl]) + opts[:room]


def hbh_packets(seed, n):
    """Ethernet (0-2 tags) / IPv6 + HopByHop / TCP or UDP, some jumbograms
    (Length 0 + Jumbo Payload, P4), some with Ethernet padding (P3)."""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        proto = rng.choice([6, 17, 59])
        jumbo = None
        if rng.randrange(6) == 0:
            jumbo = 70000 + rng.randrange(100)
        h = hbh_header(rng, proto, jumbo=jumbo)
        if proto == 6:
            l4 = struct.pack(">HHIIBBHHH", rng.randrange(65536), 443, 1, 2, 5 << 4, 0x18, 9, 0, 0)
        elif proto == 17:
            l4 = struct.pack(">HHHH", 53, rng.randrange(65536), 8 + 12, 0) + bytes(12)
        else:
            l4 = b""
        body = h + l4 + bytes(rng.randrange(40))
        length = 0 if jumbo else len(body)
        ip6 = struct.pack(">IHBB16s16s", 0x60000000 | rng.randrange(1 << 20), length, 0, 64,
                          bytes(rng.randrange(256) for _ in range(16)), bytes(rng.randrange(256) for _ in range(16)))
        tags = b""
        for _ in range(rng.choice([0, 0, 1, 2])):
            tags += struct.pack(">HH", rng.randrange(65536) & 0xEFFF, 0)
        eth = bytes(12)
        if tags:
            parts = [tags[i:i + 4] for i in range(0, len(tags), 4)]
            eth += b"\x81\x00"
            for k, t in enumerate(parts):
                eth += t[:2] + (b"\x81\x00" if k + 1 < len(parts) else b"\x86\xdd")
        else:
            eth += b"\x86\xdd"
        pad = bytes(rng.randrange(12)) if rng.randrange(3) == 0 else b""
        out.append(eth + ip6 + body + pad)
    return out


def strip_ethernet(p):
    """The bytes after the Ethernet header and its tags."""
    off = 12
    while p[off:off + 2] == b"\x81\x00":
        off += 4
    return p[off + 2:]


def state(x, depth=0):
    """A layer struct as plain data (nested structs included), for equality."""
    if depth > 4:
        return None
    if isinstance(x, (G.Payload, L.BaseLayer, L.IPv6HopByHop)):
        return (type(x).__name__, {k: state(v, depth + 1) for k, v in sorted(vars(x).items()) if k != "_poff"})
    if isinstance(x, list):
        return [state(v, depth + 1) for v in x]
    if isinstance(x, (bytes, bytearray, memoryview)):
        return bytes(x)
    return x


DECODERS = (L.Ethernet, L.Dot1Q, L.IPv4, L.IPv6, L.IPv6ExtensionSkipper, L.TCP, L.UDP, G.Payload)


def parser(decoders=DECODERS, first=17):
    return G.DecodingLayerParser(G.LayerType(first), *[d() for d in decoders])


def compare(res_a, res_b, pa, pb, indices):
    """Hydrate packet after packet from two results of the same batch into two
    parsers (each keeps its structs' state across packets, as the reference's
    reused structs do); every decoded list, error, Truncated flag and struct
    must agree. Returns the number of packets compared."""
    n = 0
    for i in indices:
        da, db = [], []
        ea, eb = res_a.Hydrate(i, da), res_b.Hydrate(i, db)
        assert da == db, i
        assert ea == eb, (i, ea, eb)
        assert pa.Truncated == pb.Truncated, i
        for k in pa._decoders:
            sa, sb = state(pa._decoders[k]), state(pb._decoders[k])
            assert sa == sb, (i, k, sa, sb)
        n += 1
    return n


def oracle_results(p, batch, decoders):
    """BatchResult pair from the oracle (tests only): one with layouts, one
    with the fields record and no layouts."""
    from oracle import oracle as O
    names = {L.Ethernet: "ETHERNET", L.Dot1Q: "DOT1Q", L.IPv4: "IPV4", L.IPv6: "IPV6",
             L.IPv6ExtensionSkipper: "IPV6_EXT", L.TCP: "TCP", L.UDP: "UDP", G.Payload: "PAYLOAD",
             G.Fragment: "FRAGMENT"}
    r = O.OracleParser(int(p.first), [names[d] for d in decoders]).decode(batch.data, batch.offsets, batch.caplens)
    f = O.extract_fields(batch.data, batch.offsets, r["layouts"]).view(_lib.FIELDS_DTYPE).reshape(-1)
    with_layouts = G.BatchResult(p, batch, dict(r))
    rf = dict(r)
    rf["layouts"] = None
    with_fields = G.BatchResult(p, batch, rf)
    with_fields.fields = f
    return with_layouts, with_fields, r
