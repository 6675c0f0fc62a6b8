"""AF_PACKET ring builder for tests: TPACKET_V1/V2 frame rings and TPACKET_V3
block rings with the kernel's layout (pinned by the live captures in
tests/golden/afpacket/: V3 tp_mac 82 / tp_net 96, V1/V2 tp_mac 66 / tp_net 80,
sockaddr_ll after the aligned header), plus knobs the kernel never turns
(zero next offsets, empty blocks, stale lengths, out-of-ring chains) so the
walker's handling of them can be compared with the oracle's.
"""
import struct

ALIGN = 16


def al(x):
    return (x + ALIGN - 1) & ~(ALIGN - 1)


def _sll(buf, p, ifindex, proto=0x0008):
    struct.pack_into("<HHiHBB8s", buf, p, 17, proto, ifindex, 1, 0, 6, b"\x02\x00\x00\x00\x00\x01\x00\x00")


def v3_ring(blocks, block_size, num_blocks):
    """blocks[b] = dict(status, pkts=[dict(data, length=None, sec, nsec, pstatus=1, tci=0, mac=82,
    next='auto'|'zero'|int)], num_pkts=None, o2fp=48, ifindex=2)."""
    ring = bytearray(block_size * num_blocks)
    for b, blk in enumerate(blocks):
        base = b * block_size
        o2fp = blk.get("o2fp", 48)
        pkts = blk.get("pkts", [])
        pos = o2fp
        for k, pk in enumerate(pkts):
            d = pk["data"]
            mac = pk.get("mac", 82)
            step = al(mac + len(d))
            nx = pk.get("next", "auto")
            nxv = step if nx == "auto" else (0 if nx == "zero" else int(nx))
            if k + 1 == len(pkts) and nx == "auto":
                nxv = 0
            p = base + pos
            if p + mac + len(d) > base + block_size:
                raise ValueError("block overflow")
            length = pk.get("length", len(d))
            struct.pack_into("<IIIIIIHH", ring, p, nxv, pk.get("sec", 1700000000 + k), pk.get("nsec", k * 1000),
                             len(d), length, pk.get("pstatus", 1), mac, mac + 14)
            struct.pack_into("<IIH", ring, p + 28, pk.get("rxhash", 0), pk.get("tci", 0), pk.get("tpid", 0))
            _sll(ring, p + 48, blk.get("ifindex", 2))
            ring[p + mac:p + mac + len(d)] = d
            pos += step  # the layout; an explicit next offset only changes the chain
        n = blk.get("num_pkts", len(pkts))
        struct.pack_into("<IIIIIIQ", ring, base, 2, 48, blk.get("status", 1), n, o2fp, pos, b + 1)
    return ring


def frame_ring(version, frames, frame_size, nframes):
    """frames[f] = dict(status, data, length=None, sec, frac (usec for V1, nsec for V2), tci=0, mac=66)."""
    ring = bytearray(frame_size * nframes)
    for f, fr in enumerate(frames):
        p = f * frame_size
        d = fr.get("data", b"")
        mac = fr.get("mac", 66)
        length = fr.get("length", len(d))
        if version == 0:
            struct.pack_into("<QIIHHII", ring, p, fr.get("status", 1), length, len(d), mac, mac + 14,
                             fr.get("sec", 1700000000 + f), fr.get("frac", f))
        else:
            struct.pack_into("<IIIHHIIHH", ring, p, fr.get("status", 1), length, len(d), mac, mac + 14,
                             fr.get("sec", 1700000000 + f), fr.get("frac", f * 1000), fr.get("tci", 0),
                             fr.get("tpid", 0))
        _sll(ring, p + 32, fr.get("ifindex", 3))
        if p + mac + len(d) <= len(ring):
            ring[p + mac:p + mac + len(d)] = d
    return ring


def random_packet(rng, lo=0, hi=300):
    n = int(rng.integers(lo, hi + 1))
    return bytes(rng.integers(0, 256, n, dtype=int).astype("uint8"))


def random_v3(rng, block_size=4096, num_blocks=6):
    blocks = []
    for b in range(num_blocks):
        r = rng.random()
        status = 1 if r < 0.7 else (0 if r < 0.85 else 0x21)
        pkts = []
        room = block_size - 48
        for _ in range(int(rng.integers(0, 12))):
            pk = dict(data=random_packet(rng, 0 if rng.random() < 0.1 else 14, 260),
                      sec=int(rng.integers(0, 1 << 32)), nsec=int(rng.integers(0, 1 << 32)),
                      pstatus=int(rng.choice([1, 9, 0x11, 0x19])),
                      tci=int(rng.choice([0, 0, 5, 0x1FFF, 0x12345])))
            if rng.random() < 0.1:
                pk["length"] = 0
            if rng.random() < 0.15:
                pk["next"] = "zero"
            if rng.random() < 0.05:
                pk["mac"] = 98
            step = al(pk.get("mac", 82) + len(pk["data"]))
            if step > room:
                break
            room -= step
            pkts.append(pk)
        blk = dict(status=status, pkts=pkts)
        if rng.random() < 0.08:
            blk["num_pkts"] = len(pkts) + int(rng.integers(1, 3))  # more than written: the chain runs on
        blocks.append(blk)
    return v3_ring(blocks, block_size, num_blocks)


def random_frames(rng, version, frame_size=512, nframes=16):
    frames = []
    for f in range(nframes):
        r = rng.random()
        d = random_packet(rng, 0 if rng.random() < 0.1 else 14, frame_size - 66)
        fr = dict(status=1 if r < 0.75 else (0 if r < 0.9 else 5), data=d, sec=int(rng.integers(0, 1 << 32)),
                  frac=int(rng.integers(0, 1 << 32)), tci=int(rng.choice([0, 0, 7, 0xFFFF])))
        if rng.random() < 0.1:
            fr["length"] = 0
        frames.append(fr)
    return frame_ring(version, frames, frame_size, nframes)
