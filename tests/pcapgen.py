"""Small pcap / pcapng writers for tests (our own, from the file-format layout;
nothing here is copied from the reference). Used to build edge-case captures
and fuzz inputs for the pcapgo reader parity tests."""
import struct


def _pad4(b):
    return b + b"\x00" * ((4 - len(b) % 4) % 4)


def opt(code, value, bo="<"):
    return struct.pack(bo + "HH", code, len(value)) + _pad4(value)


def end_opt(bo="<"):
    return struct.pack(bo + "HH", 0, 0)


def block(typ, body, bo="<", total=None):
    n = 12 + len(body) if total is None else total
    return struct.pack(bo + "II", typ, n) + body + struct.pack(bo + "I", n)


def shb(bo="<", options=b"", major=1, minor=0, section_len=-1):
    body = struct.pack(bo + "IHHq", 0x1A2B3C4D, major, minor, section_len) + options
    return block(0x0A0D0D0A, body, bo)


def idb(link_type=1, snaplen=0, bo="<", options=b""):
    return block(1, struct.pack(bo + "HHI", link_type, 0, snaplen) + options, bo)


def epb(data, iface=0, ts=0, length=None, bo="<", options=b"", caplen=None):
    cl = len(data) if caplen is None else caplen
    ln = len(data) if length is None else length
    body = struct.pack(bo + "IIIII", iface, ts >> 32, ts & 0xFFFFFFFF, cl, ln) + _pad4(data) + options
    return block(6, body, bo)


def spb(data, length=None, bo="<"):
    ln = len(data) if length is None else length
    return block(3, struct.pack(bo + "I", ln) + _pad4(data), bo)


def pb(data, iface=0, ts=0, length=None, bo="<"):
    ln = len(data) if length is None else length
    body = struct.pack(bo + "HHIIII", iface, 0, ts >> 32, ts & 0xFFFFFFFF, len(data), ln) + _pad4(data)
    return block(2, body, bo)


def isb(iface, ts, bo="<", options=b""):
    return block(5, struct.pack(bo + "III", iface, ts >> 32, ts & 0xFFFFFFFF) + options, bo)


def nrb(records, bo="<"):
    """records: list of (type, value bytes)."""
    body = b"".join(struct.pack(bo + "HH", t, len(v)) + _pad4(v) for t, v in records)
    return block(4, body + struct.pack(bo + "HH", 0, 0), bo)


def dsb(secret_type, payload, bo="<"):
    return block(0xA, struct.pack(bo + "II", secret_type, len(payload)) + _pad4(payload), bo)


def ng_file(packets, bo="<", link_type=1, snaplen=0):
    return shb(bo) + idb(link_type, snaplen, bo) + b"".join(epb(p, ts=i * 1000, bo=bo) for i, p in enumerate(packets))


def pcap_file(packets, bo="<", nano=False, snaplen=65535, link_type=1):
    magic = 0xA1B23C4D if nano else 0xA1B2C3D4
    out = [struct.pack(bo + "IHHiIII", magic, 2, 4, 0, 0, snaplen, link_type)]
    for i, p in enumerate(packets):
        out.append(struct.pack(bo + "IIII", 1400000000 + i, i * 7, len(p), len(p) + (i % 3)) + p)
    return b"".join(out)
