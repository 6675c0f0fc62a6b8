"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg. The product package gopacket_amd never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

RECORD_DTYPE = np.dtype([("layers", "<u8"), ("status", "<u4"), ("ip4_csum", "<u2"), ("l4_csum", "<u2")])
LAYOUT_DTYPE = np.dtype([("start", "<u4", (8,)), ("end", "<u4", (8,))])
RECORD8_DTYPE = np.dtype([("layers", "<u4"), ("status", "<u4")])  # include/gpk.h gpk_record8

FIELDS_ITEMSIZE = 128  # include/gpk.h gpk_fields

# decoder kinds (include/gpk.h GPK_DEC_*)
DEC = dict(ETHERNET=1, DOT1Q=2, IPV4=3, IPV6=4, IPV6_EXT=5, TCP=6, UDP=7, PAYLOAD=8, FRAGMENT=9)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_sizeof_config.restype = ctypes.c_uint64
        L.oracle_config_init.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.oracle_config_put.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.oracle_decode_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_decode_batch_narrow.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_decoded_list.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                          ctypes.c_void_p, ctypes.c_uint32]
        L.oracle_decoded_list.restype = ctypes.c_uint32
        L.oracle_error_string.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_char_p, ctypes.c_int]
        L.oracle_compute_checksum.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_compute_checksum.restype = ctypes.c_uint32
        L.oracle_fold_checksum.argtypes = [ctypes.c_uint32]
        L.oracle_fold_checksum.restype = ctypes.c_uint16
        L.oracle_fnv_hash.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
        L.oracle_fnv_hash.restype = ctypes.c_uint64
        L.oracle_flow_fast_hash.argtypes = [ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint32,
                                            ctypes.c_char_p, ctypes.c_uint32]
        L.oracle_flow_fast_hash.restype = ctypes.c_uint64
        L.oracle_config_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint32]
        L.oracle_config_table.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.oracle_config_table.restype = ctypes.c_void_p
        _LIB = L
    return _LIB


class OracleParser:
    """The oracle's view of a DecodingLayerParser configuration."""

    def __init__(self, first, decoders, ignore_unsupported=False, ignore_panic=False, outputs=7,
                 ethertype=None, ipprotocol=None, tcp_port=None, udp_port=None):
        L = lib()
        self._buf = ctypes.create_string_buffer(int(L.oracle_sizeof_config()))
        self.ptr = ctypes.cast(self._buf, ctypes.c_void_p)
        L.oracle_config_init(self.ptr, int(first))
        for d in decoders:
            L.oracle_config_put(self.ptr, DEC[d] if isinstance(d, str) else int(d))
        L.oracle_config_set(self.ptr, int(bool(ignore_unsupported)), int(bool(ignore_panic)), int(outputs))
        for which, (count, over) in enumerate(((65536, ethertype), (256, ipprotocol),
                                              (65536, tcp_port), (65536, udp_port))):
            if over:
                arr = (ctypes.c_int32 * count).from_address(L.oracle_config_table(self.ptr, which))
                for k, v in over.items():
                    arr[int(k)] = int(v)

    def decode(self, data, offsets, caplens, nthreads=1, layouts=True):
        L = lib()
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        caplens = np.ascontiguousarray(caplens, dtype=np.uint32)
        n = len(offsets)
        rec = np.zeros(n, RECORD_DTYPE)
        err = np.zeros(2 * n, np.uint32)
        flows = np.zeros(3 * n, np.uint64)
        lay = np.zeros(n, LAYOUT_DTYPE) if layouts else None
        L.oracle_decode_batch(self.ptr, data.ctypes.data, offsets.ctypes.data, caplens.ctypes.data, n,
                              rec.ctypes.data, err.ctypes.data, flows.ctypes.data,
                              lay.ctypes.data if layouts else None, int(nthreads))
        return dict(records=rec, err_args=err, flows=flows, layouts=lay)

    def decode_narrow(self, data, offsets, caplens, nthreads=1):
        """The narrow form (gpk_decode_batch_narrow): records8 (RECORD8_DTYPE)
        and the side array wide (RECORD_DTYPE, zero except where a record8 has
        GPK_ST8_WIDE), err_args, flows."""
        L = lib()
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        caplens = np.ascontiguousarray(caplens, dtype=np.uint32)
        n = len(offsets)
        rec8 = np.zeros(n, RECORD8_DTYPE)
        wide = np.zeros(n, RECORD_DTYPE)
        err = np.zeros(2 * n, np.uint32)
        flows = np.zeros(3 * n, np.uint64)
        L.oracle_decode_batch_narrow(self.ptr, data.ctypes.data, offsets.ctypes.data, caplens.ctypes.data, n,
                                     rec8.ctypes.data, wide.ctypes.data, err.ctypes.data, flows.ctypes.data,
                                     int(nthreads))
        return dict(records8=rec8, wide=wide, err_args=err, flows=flows)

    def decoded_list(self, pkt):
        L = lib()
        pkt = bytes(pkt)
        out = (ctypes.c_int64 * 4096)()
        n = L.oracle_decoded_list(self.ptr, pkt, len(pkt), out, 4096)
        return [out[i] for i in range(min(n, 4096))]

    def error_string(self, code, a0=0, a1=0):
        buf = ctypes.create_string_buffer(512)
        lib().oracle_error_string(self.ptr, int(code), int(a0) & 0xFFFFFFFF, int(a1) & 0xFFFFFFFF, buf, 512)
        return buf.value.decode()


def compute_checksum(data, csum=0):
    data = bytes(data)
    return lib().oracle_compute_checksum(data, len(data), csum)


def fold_checksum(csum):
    return lib().oracle_fold_checksum(csum)


def fnv_hash(s):
    s = bytes(s)
    return lib().oracle_fnv_hash(s, len(s))


def flow_fast_hash(typ, src, dst):
    src, dst = bytes(src), bytes(dst)
    return lib().oracle_flow_fast_hash(typ, src, len(src), dst, len(dst))


BPF_INSN_DTYPE = np.dtype([("code", "<u2"), ("jt", "u1"), ("jf", "u1"), ("k", "<u4")])


def bpf_program(insns):
    arr = np.zeros(len(insns), BPF_INSN_DTYPE)
    for i, x in enumerate(insns):
        arr[i] = (int(x[0]) & 0xFFFF, int(x[1]) & 0xFF, int(x[2]) & 0xFF, int(x[3]) & 0xFFFFFFFF)
    return arr


def bpf_filter(insns, pkt, wirelen=None):
    """libpcap bpf_filter restated (oracle/bpf_oracle.c): the filter's return value."""
    L = lib()
    prog = bpf_program(insns)
    pkt = bytes(pkt)
    L.oracle_bpf_filter.restype = ctypes.c_uint32
    L.oracle_bpf_filter.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
                                    ctypes.c_uint32]
    return L.oracle_bpf_filter(prog.ctypes.data, len(prog), pkt, len(pkt) if wirelen is None else wirelen, len(pkt))


def bpf_batch(insns, data, offsets, caplens, wirelens=None):
    L = lib()
    prog = bpf_program(insns)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    caplens = np.ascontiguousarray(caplens, dtype=np.uint32)
    w = None if wirelens is None else np.ascontiguousarray(wirelens, dtype=np.uint32)
    ret = np.zeros(len(offsets), np.uint32)
    L.oracle_bpf_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    L.oracle_bpf_batch(prog.ctypes.data, len(prog), data.ctypes.data, offsets.ctypes.data, caplens.ctypes.data,
                       w.ctypes.data if w is not None else None, len(offsets), ret.ctypes.data)
    return ret


def extract_fields(data, offsets, layouts):
    """oracle_extract_fields: the gpk_fields records (raw bytes, n x 128) of the
    packets from the layouts of a decode."""
    L = lib()
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    layouts = np.ascontiguousarray(layouts)
    n = len(offsets)
    out = np.zeros((n, FIELDS_ITEMSIZE), np.uint8)
    L.oracle_extract_fields.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.c_void_p]
    L.oracle_extract_fields(data.ctypes.data, offsets.ctypes.data, layouts.ctypes.data, n, out.ctypes.data)
    return out


def group_batch(kind, data, offsets, records, layouts, flows=None, buckets=8):
    """oracle/flows_oracle.c: (number of groups, group_of per packet)."""
    L = lib()
    n = len(offsets)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    out = np.zeros(n, np.int32)
    L.oracle_group_batch.restype = ctypes.c_int64
    L.oracle_group_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
    g = L.oracle_group_batch(int(kind), data.ctypes.data, offsets.ctypes.data, records.ctypes.data,
                             layouts.ctypes.data if layouts is not None else None,
                             flows.ctypes.data if flows is not None else None, n, buckets, out.ctypes.data)
    return g, out
