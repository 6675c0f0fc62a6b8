#!/usr/bin/env python3
"""Capture real kernel-filled AF_PACKET rings on the loopback interface and
store them as fixtures (tests/golden/afpacket/): the ring bytes exactly as the
Linux kernel laid them out, plus the datagrams that were sent.

These pin the header layouts the ring walker and its oracle assume
(afpacket/header.go:59-137) to what the kernel actually writes. Needs
CAP_NET_RAW (root in this container); plain Python sockets, no product code.

    python tools/capture_afpacket_fixture.py
"""
import json
import mmap
import os
import socket
import struct
import time

SOL_PACKET, PACKET_VERSION, PACKET_RX_RING = 263, 10, 5
ETH_P_ALL = 3
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "afpacket")


def capture(version, block_size, block_nr, frame_size, payloads, port):
    s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(ETH_P_ALL))
    s.bind(("lo", 0))
    s.setsockopt(SOL_PACKET, PACKET_VERSION, version)
    frame_nr = block_size // frame_size * block_nr
    if version == 2:
        req = struct.pack("7I", block_size, block_nr, frame_size, frame_nr, 10, 0, 0)  # retire after 10 ms
    else:
        req = struct.pack("4I", block_size, block_nr, frame_size, frame_nr)
    s.setsockopt(SOL_PACKET, PACKET_RX_RING, req)
    total = block_size * block_nr
    ring = mmap.mmap(s.fileno(), total, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    u = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    for p in payloads:
        u.sendto(p, ("127.0.0.1", port))
    time.sleep(0.1)  # let the block retire timer hand the open V3 block over
    data = bytes(ring[:total])
    ring.close()
    s.close()
    u.close()
    return data


def main():
    os.makedirs(OUT, exist_ok=True)
    payloads = [bytes((i * 7 + j) & 0xFF for j in range(n)) for i, n in enumerate((1, 18, 100, 333, 700, 1400))]
    meta = {"payloads_hex": [p.hex() for p in payloads], "dst": "127.0.0.1", "rings": []}
    for version, bs, bn, fs, port in ((2, 4096, 4, 2048, 40001), (1, 4096, 8, 2048, 40002), (0, 4096, 8, 2048, 40003)):
        ring = capture(version, bs, bn, fs, payloads, port)
        name = "lo_v%d.ring" % (version + 1)
        with open(os.path.join(OUT, name), "wb") as f:
            f.write(ring)
        meta["rings"].append(dict(file=name, version=version, block_size=bs, num_blocks=bn, frame_size=fs,
                                  udp_port=port))
    with open(os.path.join(OUT, "lo_rings.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
