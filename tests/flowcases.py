"""Packets for the flow-keyed grouping tests (row (f)3): ip4defrag's own test
frames, frames built from the field values of its struct-based tests, and
TCP segments covering tcpassembly's "useless packet" filter."""
import json
import os
import struct

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# statsassembly + Fragment: the parser a defragmenting consumer would run
DEFRAG_PARSER = dict(first=17, decoders=["ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP", "PAYLOAD"])


def defrag_frames():
    g = json.load(open(os.path.join(GOLD, "defrag_frames.json")))
    return {k: bytes.fromhex(v) for k, v in g["frames"].items()}, g["same_datagram"]


def csum(b):
    s = 0
    for k in range(0, len(b) - 1, 2):
        s += b[k] << 8 | b[k + 1]
    if len(b) & 1:
        s += b[-1] << 8
    while s > 0xFFFF:
        s = (s >> 16) + (s & 0xFFFF)
    return ~s & 0xFFFF


def eth_ip4(src, dst, ident, flags, frag_off, length, proto=1, payload=b"", ttl=15, total=None):
    """Ethernet + IPv4 header with the given field values (Length may disagree with the bytes)."""
    ip = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0, length, ident, flags << 13 | frag_off, ttl, proto, 0,
                               bytes(src), bytes(dst)))
    struct.pack_into(">H", ip, 10, csum(ip))
    frame = b"\x00\x11\x22\x33\x44\x55\x66\x77\x88\x99\xaa\xbb\x08\x00" + bytes(ip) + payload
    if total is not None:
        frame = frame[:total] + b"\x00" * max(0, total - len(frame))
    return frame


def defrag_struct_cases():
    """(label, frame): the field values of defrag_test.go's struct-based tests."""
    a, b = (1, 1, 1, 1), (2, 2, 2, 2)
    MF, DF = 1, 2
    return [
        ("TestNotFrag (DF)", eth_ip4(a, b, 0, DF, 0, 20)),
        ("TestDefragTooSmall Length 27 MF", eth_ip4(a, b, 0xcc, MF, 0, 27, payload=b"x" * 7)),
        ("TestDefragTooSmall Length 28 MF", eth_ip4(a, b, 0xcc, MF, 0, 28, payload=b"x" * 8)),
        ("TestDefragSmallFinalFragment", eth_ip4(a, b, 0xcc, 0, 0, 27, payload=b"x" * 7)),
        ("TestDefragFragmentOffset 0", eth_ip4(a, b, 0xcc, MF, 0, 512, payload=b"y" * 492)),
        ("TestDefragFragmentOffset 8184", eth_ip4(a, b, 0xcc, MF, 8184, 512, payload=b"y" * 492)),
        ("TestDefragMaxSize Length 65535", eth_ip4(a, b, 0xcc, MF, 0, 65535, payload=b"z" * 100)),
        ("TestDefragMaxSize Length 28 off 1", eth_ip4(a, b, 0xcc, MF, 1, 28, payload=b"z" * 8)),
        ("last fragment, offset 8183", eth_ip4(a, b, 0xcd, 0, 8183, 28, payload=b"z" * 8)),
        ("TSO Length 0 with MF", eth_ip4(a, b, 0xce, MF, 0, 0, payload=b"w" * 40)),
        ("Length 0, IHL 5, short", eth_ip4(a, b, 0xcf, MF, 3, 0, payload=b"w" * 2)),
    ]


def tcp_segment(src, dst, sport, dport, flags, payload=b"", v6=False, pad=0):
    tcp = struct.pack(">HHIIBBHHH", sport, dport, 1, 0, 5 << 4, flags, 512, 0, 0) + payload
    if v6:
        ip = struct.pack(">IHBB16s16s", 0x60000000, len(tcp), 6, 64, bytes(src), bytes(dst))
        et = b"\x86\xdd"
    else:
        ip = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + len(tcp), 1, 0x4000, 64, 6, 0, bytes(src), bytes(dst)))
        struct.pack_into(">H", ip, 10, csum(ip))
        et = b"\x08\x00"
    return b"\x02\x00\x00\x00\x00\x01\x02\x00\x00\x00\x00\x02" + et + bytes(ip) + tcp + b"\x00" * pad


def connection_cases():
    a4, b4 = (10, 0, 0, 1), (10, 0, 0, 2)
    a6, b6 = bytes(range(16)), bytes(range(16, 32))
    SYN, FIN, RST, ACK, PSH = 2, 1, 4, 16, 8
    return [
        tcp_segment(a4, b4, 1000, 2000, SYN),
        tcp_segment(b4, a4, 2000, 1000, SYN | ACK),          # the other direction: its own key
        tcp_segment(a4, b4, 1000, 2000, ACK),                 # useless: no flags, no payload
        tcp_segment(a4, b4, 1000, 2000, ACK, pad=10),         # Ethernet padding is not payload
        tcp_segment(a4, b4, 1000, 2000, ACK | PSH, b"hello"),
        tcp_segment(a6, b6, 1000, 2000, ACK | PSH, b"v6 data", v6=True),
        tcp_segment(a6, b6, 1000, 2000, FIN | ACK, v6=True),
        tcp_segment(a4, b4, 1000, 2001, RST),
        tcp_segment(a4, b4, 1000, 2000, FIN | ACK),
    ]
