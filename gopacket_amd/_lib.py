"""ctypes binding of libgpk.so (the C ABI declared in include/gpk.h).

The shared library is built in-tree (gopacket_amd/libgpk.so, see
csrc/Makefile) so the GPU box loads exactly the code in this repository.
There is no fallback: if the library is missing or a call fails, an
exception is raised.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# GPK_LIB_VARIANT=<name> loads build/libgpk_<name>.so instead: compile-time
# kernel variants built by `make -C gopacket_amd/csrc variant V=<name>
# VDEFS=...` for A/B measurements (tools/ab.sh). Unset in normal use.
_VARIANT = os.environ.get("GPK_LIB_VARIANT")
LIB_PATH = (os.path.join(_HERE, "build", "libgpk_%s.so" % _VARIANT) if _VARIANT
            else os.path.join(_HERE, "libgpk.so"))
SYNTH_PATH = os.path.join(_HERE, "libgpk_synth.so")

# include/gpk.h constants
GPK_OK = 0
GPK_EINVAL, GPK_ENOMEM, GPK_EHIP, GPK_ENODEV, GPK_EUNSUPP = -1, -2, -3, -4, -5
GPK_STOPPED = 1  # a replay or ring pump ended early at gpk_stop (not an error)
OUT_IP4_CSUM, OUT_L4_CSUM, OUT_FLOWS, OUT_ALL = 1, 2, 4, 7
TABLES_AUTO, TABLES_GLOBAL = 0, 1
DEC_NONE, DEC_ETHERNET, DEC_DOT1Q, DEC_IPV4, DEC_IPV6, DEC_IPV6_EXT, DEC_TCP, DEC_UDP, DEC_PAYLOAD, \
    DEC_FRAGMENT = range(10)
ST_ERR_MASK = 0x7F
ST_TRUNCATED = 1 << 7
ST_NLAYERS_SHIFT = 8
ST_NLAYERS_MASK = 0xFFF
ST_IP4_CSUM = 1 << 20
ST_IP4_VALID = 1 << 21
ST_L4_CSUM = 1 << 22
ST_L4_VALID = 1 << 23
ST_L4_UDP = 1 << 24
ST_LINK_FLOW = 1 << 25
ST_NET_FLOW = 1 << 26
ST_NET_IPV6 = 1 << 27
ST_TRANSPORT_FLOW = 1 << 28
LAYOUT_ABSENT = 0xFFFFFFFF
MAX_INLINE_LAYERS = 16

RECORD_DTYPE = np.dtype([("layers", "<u8"), ("status", "<u4"), ("ip4_csum", "<u2"), ("l4_csum", "<u2")])
RECORD8_DTYPE = np.dtype([("layers", "<u4"), ("status", "<u4")])  # gpk_record8 (gpk_decode_batch_narrow)
ST8_NLAYERS_MASK, ST8_WIDE = 0xF, 1 << 12
LAYOUT_DTYPE = np.dtype([("start", "<u4", (8,)), ("end", "<u4", (8,))])
# include/gpk.h gpk_fields (128 B): the scalar layer fields (gpk_extract_fields)
FIELDS_DTYPE = np.dtype({
    "names": ["present", "hbh_opt_map", "eth_type", "eth_length", "eth_dst", "eth_src", "d1q_tci", "d1q_type", "ip4_version",
              "ip4_ihl", "ip4_tos", "ip4_ttl", "ip4_length", "ip4_id", "ip4_flags_frag", "ip4_protocol",
              "ip6_version", "ip4_checksum", "ip6_traffic_class", "ip6_next_header", "ip6_flow_label", "ip6_length",
              "ip6_hop_limit", "tcp_data_offset", "ip4_src", "ip4_dst", "ip6_src", "ip6_dst", "tcp_src_port",
              "tcp_dst_port", "tcp_seq", "tcp_ack", "tcp_flags", "tcp_window", "tcp_checksum", "tcp_urgent",
              "udp_src_port", "udp_dst_port", "udp_length", "udp_checksum", "ip4_start", "tcp_start",
              "ip4_opt_map", "tcp_opt_map"],
    "formats": ["u1", ("u1", (3,)), "<u2", "<u2", ("u1", (6,)), ("u1", (6,)), "<u2", "<u2", "u1", "u1", "u1", "u1", "<u2", "<u2",
                "<u2", "u1", "u1", "<u2", "u1", "u1", "<u4", "<u2", "u1", "u1", ("u1", (4,)), ("u1", (4,)),
                ("u1", (16,)), ("u1", (16,)), "<u2", "<u2", "<u4", "<u4", "<u2", "<u2", "<u2", "<u2", "<u2", "<u2",
                "<u2", "<u2", "u1", "u1", ("u1", (5,)), ("u1", (5,))],
    "offsets": [0, 1, 4, 6, 8, 14, 20, 22, 24, 25, 26, 27, 28, 30, 32, 34, 35, 36, 38, 39, 40, 44, 46, 47, 48, 52, 56, 72,
                88, 90, 92, 96, 100, 102, 104, 106, 108, 110, 112, 114, 116, 117, 118, 123],
    "itemsize": 128})
NAME_FIELDS = 2  # gpk_decode_kernel_name / gpk_decode_occupancy: the fused fields launch
TCP_FLAG_BITS = dict(FIN=1, SYN=2, RST=4, PSH=8, ACK=16, URG=32, ECE=64, CWR=128, NS=256)
# gpk_layout slot -> decoder kind (slot 7: Payload or Fragment)
LAYOUT_SLOTS = (DEC_ETHERNET, DEC_DOT1Q, DEC_IPV4, DEC_IPV6, DEC_IPV6_EXT, DEC_TCP, DEC_UDP, DEC_PAYLOAD)

# exported symbols, in include/gpk.h order
EXPORTS = (
    "gpk_parser_create", "gpk_parser_destroy", "gpk_parser_add_decoder", "gpk_parser_set_options",
    "gpk_parser_set_outputs", "gpk_parser_decoder_for", "gpk_parser_set_ethertype",
    "gpk_parser_set_ipprotocol", "gpk_parser_set_tcp_port", "gpk_parser_set_udp_port", "gpk_ctx_create",
    "gpk_ctx_destroy", "gpk_ctx_set_table_mode", "gpk_stop", "gpk_decode_batch", "gpk_decode_batch_narrow", "gpk_decode_batch_fields",
    "gpk_extract_fields",
    "gpk_decode_kernel_name", "gpk_decode_occupancy", "gpk_diag_set_buffer", "gpk_decode_batch_host", "gpk_decode_batch_host_fields",
    "gpk_decoded_list",
    "gpk_decoded_list_host", "gpk_host_alloc", "gpk_host_free", "gpk_format_error", "gpk_layer_type_name", "gpk_code_layer_type", "gpk_strerror",
    "gpk_last_hip_error", "gpk_abi_version",
    # include/gpk_capture.h
    "gpk_capreader_create", "gpk_capreader_destroy", "gpk_capreader_index", "gpk_capreader_error",
    "gpk_capreader_link_type", "gpk_capreader_pcap_header", "gpk_capreader_nsections", "gpk_capreader_section_info",
    "gpk_capreader_ninterfaces", "gpk_capreader_interface", "gpk_capreader_interface_str", "gpk_replay_file",
    "gpk_replay_file_range",
    "gpk_capreader_index_all", "gpk_capindex_free",
    "gpk_capreader_section_end_at", "gpk_capreader_nstat_events", "gpk_capreader_stat_event",
    "gpk_capreader_nnames", "gpk_capreader_name", "gpk_capreader_skip_section", "gpk_capreader_set_snaplen",
    "gpk_capreader_keep_options", "gpk_capreader_packet_options",
    # include/gpk_afpacket.h
    "gpk_tp_default_opts", "gpk_tp_check_opts", "gpk_tpacket_new", "gpk_tpacket_attach", "gpk_tpacket_close",
    "gpk_tpacket_ring", "gpk_tpacket_index", "gpk_tpacket_defer", "gpk_tpacket_set_threads", "gpk_tpacket_release_seq", "gpk_tpacket_release",
    "gpk_tpacket_take_new_headers", "gpk_tpacket_geometry", "gpk_tpacket_error", "gpk_tpacket_stats",
    "gpk_tpacket_socket_stats", "gpk_tpacket_set_bpf", "gpk_tpacket_set_fanout", "gpk_tpacket_pump",
    "gpk_tpacket_set_ebpf", "gpk_tpacket_set_promiscuous", "gpk_tpacket_write", "gpk_tpacket_init_socket_stats",
    # include/gpk_flows.h
    "gpk_grouper_create", "gpk_grouper_destroy", "gpk_group_batch", "gpk_pack_batch", "gpk_decode_group_batch",
    # include/gpk_bpf.h
    "gpk_bpf_create", "gpk_bpf_destroy", "gpk_bpf_run", "gpk_bpf_select",
)

BPF_INSN_DTYPE = np.dtype([("code", "<u2"), ("jt", "u1"), ("jf", "u1"), ("k", "<u4")])
BPF_MAX_INSNS = 4096

# include/gpk_flows.h constants
GROUP_CONNECTION, GROUP_DEFRAG, GROUP_NET_BUCKET = 1, 2, 3
GROUP_NONE, GROUP_USELESS, GROUP_FRAG_TOO_SMALL, GROUP_FRAG_OFFSET, GROUP_FRAG_OVERRUN, GROUP_UNKNOWN = \
    -1, -2, -3, -4, -5, -6


class Groups(ctypes.Structure):
    _fields_ = [("group_of", ctypes.c_void_p), ("perm", ctypes.c_void_p), ("start", ctypes.c_void_p),
                ("first", ctypes.c_void_p), ("counts", ctypes.c_void_p)]

# include/gpk_afpacket.h constants
TPACKET_V1, TPACKET_V2, TPACKET_V3, TPACKET_HIGHEST = 0, 1, 2, -1
TP_WAIT, TP_FULL, TP_ERROR = 0, 1, 2
TPINFO_DTYPE = np.dtype([("ts_sec", "<i8"), ("ts_nsec", "<u4"), ("length", "<u4"), ("iface", "<i4"),
                         ("vlan", "<i4")])


class TpOpts(ctypes.Structure):
    _fields_ = [("version", ctypes.c_int32), ("socktype", ctypes.c_int32), ("frame_size", ctypes.c_int32),
                ("block_size", ctypes.c_int32), ("num_blocks", ctypes.c_int32), ("frames_per_block", ctypes.c_int32),
                ("add_vlan_header", ctypes.c_int32), ("vnet_hdr_size", ctypes.c_int32),
                ("block_timeout_ns", ctypes.c_int64), ("poll_timeout_ns", ctypes.c_int64),
                ("protocol", ctypes.c_uint16), ("_pad", ctypes.c_uint16 * 3), ("iface", ctypes.c_char * 64)]


# gpk_tp_pump_fields_cb(user, first_packet, n, const gpk_fields*)
PUMP_FIELDS_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p)


# gpk_tp_pump_packets_cb(user, first_packet, n, const uint8_t* const* data, const uint32_t* caplens)
PUMP_PACKETS_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                   ctypes.c_void_p)


class PumpOpts(ctypes.Structure):
    _fields_ = [("batch_pkts", ctypes.c_uint64), ("max_packets", ctypes.c_uint64), ("wait", ctypes.c_int),
                ("inflight", ctypes.c_int), ("fields_cb", PUMP_FIELDS_CB), ("packets_cb", PUMP_PACKETS_CB)]


class PumpStats(ctypes.Structure):
    _fields_ = [("packets", ctypes.c_uint64), ("packet_bytes", ctypes.c_uint64), ("batches", ctypes.c_uint64),
                ("ring_bytes_copied", ctypes.c_uint64), ("waits", ctypes.c_uint64), ("wall_s", ctypes.c_double),
                ("index_s", ctypes.c_double), ("gpu_s", ctypes.c_double), ("kernel_s", ctypes.c_double),
                ("status", ctypes.c_int), ("error", ctypes.c_char * 160), ("kernel", ctypes.c_char * 96)]


PUMP_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p)

# include/gpk_capture.h constants
CAP_PCAP, CAP_PCAPNG = 1, 2
NG_WANT_MIXED_LINKTYPE, NG_ERROR_ON_MISMATCHING_LINKTYPE, NG_SKIP_UNKNOWN_VERSION = 1, 2, 4
CAP_MORE, CAP_FULL, CAP_END = 0, 1, 2
CAPINFO_DTYPE = np.dtype([("ts_sec", "<i8"), ("ts_nsec", "<u4"), ("length", "<u4"), ("iface", "<i4"),
                          ("link_type", "<i4")])


class CapIndex(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("offsets", ctypes.c_void_p), ("caplens", ctypes.c_void_p),
                ("ci", ctypes.c_void_p)]


class NgInterface(ctypes.Structure):
    _fields_ = [("link_type", ctypes.c_uint16), ("ts_resolution", ctypes.c_uint8),
                ("has_statistics", ctypes.c_uint8), ("snap_length", ctypes.c_uint32), ("ts_offset", ctypes.c_uint64),
                ("last_update_sec", ctypes.c_int64), ("start_time_sec", ctypes.c_int64),
                ("end_time_sec", ctypes.c_int64), ("last_update_nsec", ctypes.c_uint32),
                ("start_time_nsec", ctypes.c_uint32), ("end_time_nsec", ctypes.c_uint32), ("_pad", ctypes.c_uint32),
                ("packets_received", ctypes.c_uint64), ("packets_dropped", ctypes.c_uint64)]


# gpk_replay_fields_cb(user, first_packet, n, const gpk_fields*)
REPLAY_FIELDS_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p)
# gpk_replay_packets_cb(user, first_packet, n, base, bytes, offsets, caplens)
REPLAY_PACKETS_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p)


class ReplayOpts(ctypes.Structure):
    _fields_ = [("format", ctypes.c_int), ("ng_flags", ctypes.c_uint32), ("slot_bytes", ctypes.c_uint64),
                ("slots", ctypes.c_int), ("batch_pkts", ctypes.c_uint64), ("read_threads", ctypes.c_int),
                ("fields_cb", REPLAY_FIELDS_CB), ("packets_cb", REPLAY_PACKETS_CB)]


class ReplayStats(ctypes.Structure):
    _fields_ = [("packets", ctypes.c_uint64), ("packet_bytes", ctypes.c_uint64), ("file_bytes", ctypes.c_uint64),
                ("stream_bytes", ctypes.c_uint64), ("batches", ctypes.c_uint64), ("slots", ctypes.c_uint64),
                ("wall_s", ctypes.c_double), ("read_s", ctypes.c_double), ("index_s", ctypes.c_double),
                ("gpu_s", ctypes.c_double), ("kernel_s", ctypes.c_double), ("deliver_s", ctypes.c_double),
                ("reader_status", ctypes.c_int), ("error", ctypes.c_char * 160), ("kernel", ctypes.c_char * 96),
                ("device_walk_packets", ctypes.c_uint64), ("alloc_wait_s", ctypes.c_double)]


class ReplayRange(ctypes.Structure):
    _fields_ = [("begin", ctypes.c_uint64), ("end", ctypes.c_uint64), ("header_end", ctypes.c_uint64),
                ("sync_begin", ctypes.c_uint64), ("sync_end", ctypes.c_uint64), ("clean", ctypes.c_int),
                ("state_changed", ctypes.c_int)]


REPLAY_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p)


class GpkError(RuntimeError):
    """A negative status from the C ABI."""


class Batch(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("caplens", ctypes.c_void_p),
                ("n", ctypes.c_uint64), ("data_bytes", ctypes.c_uint64)]


class Results(ctypes.Structure):
    _fields_ = [("records", ctypes.c_void_p), ("err_args", ctypes.c_void_p), ("flows", ctypes.c_void_p),
                ("layouts", ctypes.c_void_p)]


class Results8(ctypes.Structure):
    _fields_ = [("records", ctypes.c_void_p), ("wide", ctypes.c_void_p), ("err_args", ctypes.c_void_p),
                ("flows", ctypes.c_void_p)]


_lib = None


def _share_hip_runtime():
    """One HIP runtime per process. PyTorch-ROCm ships its own libamdhip64
    (SONAME libamdhip64.so.7, NEEDED as "libamdhip64.so" by libtorch_hip), so
    if libgpk.so were loaded first the process would end up with two HIP/HSA
    runtimes and the second one finds no device. Importing torch first makes
    libgpk's libamdhip64.so.7 resolve to torch's already-loaded copy."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("gopacket_amd: %s is not built (run __graft_entry__.build() or make -C "
                          "gopacket_amd/csrc)" % LIB_PATH)
    _share_hip_runtime()
    L = ctypes.CDLL(LIB_PATH)
    vp, i64, u32, u64, c_int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    P = ctypes.POINTER
    sig = {
        "gpk_parser_create": ([P(vp), i64], c_int),
        "gpk_parser_destroy": ([vp], c_int),
        "gpk_parser_add_decoder": ([vp, c_int], c_int),
        "gpk_parser_set_options": ([vp, c_int, c_int], c_int),
        "gpk_parser_set_outputs": ([vp, u32], c_int),
        "gpk_parser_decoder_for": ([vp, i64], c_int),
        "gpk_parser_set_ethertype": ([vp, u32, ctypes.c_int32], c_int),
        "gpk_parser_set_ipprotocol": ([vp, u32, ctypes.c_int32], c_int),
        "gpk_parser_set_tcp_port": ([vp, u32, ctypes.c_int32], c_int),
        "gpk_parser_set_udp_port": ([vp, u32, ctypes.c_int32], c_int),
        "gpk_ctx_create": ([P(vp), c_int], c_int),
        "gpk_ctx_destroy": ([vp], c_int),
        "gpk_ctx_set_table_mode": ([vp, c_int], c_int),
        "gpk_stop": ([vp], c_int),
        "gpk_decode_batch": ([vp, vp, P(Batch), P(Results), vp], c_int),
        "gpk_decode_batch_narrow": ([vp, vp, P(Batch), P(Results8), vp], c_int),
        "gpk_decode_batch_host": ([vp, vp, P(Batch), P(Results)], c_int),
        "gpk_decode_batch_host_fields": ([vp, vp, P(Batch), P(Results), vp], c_int),
        "gpk_extract_fields": ([P(Batch), vp, vp, vp], c_int),
        "gpk_decode_batch_fields": ([vp, vp, P(Batch), P(Results), vp, vp], c_int),
        "gpk_decode_kernel_name": ([vp, vp, P(Batch), c_int, ctypes.c_char_p, ctypes.c_size_t], c_int),
        "gpk_decode_occupancy": ([vp, vp, P(Batch), c_int, P(c_int)], c_int),
        "gpk_diag_set_buffer": ([vp], c_int),
        "gpk_decoded_list": ([vp, vp, P(Batch), u64, P(i64), u32, P(u32)], c_int),
        "gpk_decoded_list_host": ([vp, vp, ctypes.c_char_p, u32, P(i64), u32, P(u32)], c_int),
        "gpk_host_alloc": ([P(vp), ctypes.c_size_t], c_int),
        "gpk_host_free": ([vp], c_int),
        "gpk_format_error": ([ctypes.c_uint, u32, u32, ctypes.c_char_p, ctypes.c_size_t], c_int),
        "gpk_layer_type_name": ([i64, ctypes.c_char_p, ctypes.c_size_t], c_int),
        "gpk_code_layer_type": ([ctypes.c_uint], i64),
        "gpk_strerror": ([c_int], ctypes.c_char_p),
        "gpk_last_hip_error": ([], ctypes.c_char_p),
        "gpk_abi_version": ([], c_int),
        "gpk_capreader_create": ([P(vp), c_int, u32], c_int),
        "gpk_capreader_destroy": ([vp], c_int),
        "gpk_capreader_index": ([vp, vp, u64, c_int, vp, vp, vp, u64, P(u64), P(u64)], c_int),
        "gpk_capreader_error": ([vp, ctypes.c_char_p, ctypes.c_size_t, P(c_int), P(c_int)], c_int),
        "gpk_capreader_link_type": ([vp], c_int),
        "gpk_capreader_pcap_header": ([vp, P(u32), P(ctypes.c_uint16), P(ctypes.c_uint16), P(c_int)], c_int),
        "gpk_capreader_nsections": ([vp], c_int),
        "gpk_capreader_section_info": ([vp, c_int, c_int, ctypes.c_char_p, ctypes.c_size_t], c_int),
        "gpk_capreader_ninterfaces": ([vp, c_int], c_int),
        "gpk_capreader_interface": ([vp, c_int, c_int, P(NgInterface)], c_int),
        "gpk_capreader_interface_str": ([vp, c_int, c_int, c_int, ctypes.c_char_p, ctypes.c_size_t], c_int),
        "gpk_capreader_section_end_at": ([vp, c_int, P(ctypes.c_uint64), P(ctypes.c_uint64)], c_int),
        "gpk_capreader_nstat_events": ([vp], c_int),
        "gpk_capreader_stat_event": ([vp, c_int, P(ctypes.c_uint64), P(ctypes.c_uint64), P(c_int), P(NgInterface),
                                      ctypes.c_char_p, ctypes.c_size_t], c_int),
        "gpk_capreader_nnames": ([vp], c_int),
        "gpk_capreader_name": ([vp, c_int, P(c_int), vp, P(c_int), P(c_int), ctypes.c_char_p, ctypes.c_size_t],
                               c_int),
        "gpk_capreader_skip_section": ([vp], c_int),
        "gpk_capreader_set_snaplen": ([vp, ctypes.c_uint32], c_int),
        "gpk_capreader_keep_options": ([vp, c_int], c_int),
        "gpk_capreader_packet_options": ([vp, ctypes.c_uint64, P(vp), P(ctypes.c_uint64)], c_int),
        "gpk_replay_file": ([vp, vp, ctypes.c_char_p, P(ReplayOpts), REPLAY_CB, vp, P(ReplayStats)], c_int),
        "gpk_replay_file_range": ([vp, vp, ctypes.c_char_p, P(ReplayRange), P(ReplayOpts), REPLAY_CB, vp,
                                   P(ReplayStats)], c_int),
        "gpk_capreader_index_all": ([vp, vp, u64, c_int, c_int, P(CapIndex), P(u64)], c_int),
        "gpk_capindex_free": ([P(CapIndex)], c_int),
        "gpk_tp_default_opts": ([P(TpOpts)], None),
        "gpk_tp_check_opts": ([P(TpOpts), ctypes.c_char_p, ctypes.c_size_t], c_int),
        "gpk_tpacket_new": ([P(vp), P(TpOpts), ctypes.c_char_p, ctypes.c_size_t], c_int),
        "gpk_tpacket_attach": ([P(vp), vp, u64, c_int, P(TpOpts)], c_int),
        "gpk_tpacket_close": ([vp], c_int),
        "gpk_tpacket_ring": ([vp, P(vp), P(u64), P(c_int), P(c_int)], c_int),
        "gpk_tpacket_index": ([vp, c_int, vp, vp, vp, u64, P(u64), vp, u64, P(u64)], c_int),
        "gpk_tpacket_defer": ([vp, c_int], c_int),
        "gpk_tpacket_set_threads": ([vp, c_int], c_int),
        "gpk_tpacket_release_seq": ([vp, P(u64)], c_int),
        "gpk_tpacket_release": ([vp, u64], c_int),
        "gpk_tpacket_take_new_headers": ([vp, P(u64), P(u64)], c_int),
        "gpk_tpacket_geometry": ([vp, P(u64), P(u64)], c_int),
        "gpk_tpacket_error": ([vp, ctypes.c_char_p, ctypes.c_size_t, P(c_int)], c_int),
        "gpk_tpacket_stats": ([vp, P(i64), P(i64)], c_int),
        "gpk_tpacket_socket_stats": ([vp, P(u32), P(u32), P(u32)], c_int),
        "gpk_tpacket_set_bpf": ([vp, vp, u32], c_int),
        "gpk_tpacket_set_fanout": ([vp, c_int, ctypes.c_uint16], c_int),
        "gpk_tpacket_set_ebpf": ([vp, ctypes.c_int32], c_int),
        "gpk_tpacket_set_promiscuous": ([vp, c_int], c_int),
        "gpk_tpacket_write": ([vp, vp, ctypes.c_uint64], c_int),
        "gpk_tpacket_init_socket_stats": ([vp], c_int),
        "gpk_tpacket_pump": ([vp, vp, vp, P(PumpOpts), PUMP_CB, vp, P(PumpStats)], c_int),
        "gpk_grouper_create": ([P(vp), c_int, u64], c_int),
        "gpk_grouper_destroy": ([vp], c_int),
        "gpk_group_batch": ([vp, P(Batch), P(Results), c_int, u32, P(Groups), vp], c_int),
        "gpk_pack_batch": ([P(Batch), vp, u64, vp, vp, vp, vp], c_int),
        "gpk_decode_group_batch": ([vp, vp, P(Batch), P(Results), vp, c_int, P(Groups), vp], c_int),
        "gpk_bpf_create": ([P(vp), vp, u32, ctypes.c_char_p, ctypes.c_size_t], c_int),
        "gpk_bpf_destroy": ([vp], c_int),
        "gpk_bpf_run": ([vp, P(Batch), vp, vp, vp], c_int),
        "gpk_bpf_select": ([vp, P(Batch), vp, vp, vp, vp, vp, vp], c_int),
    }
    for name, (args, res) in sig.items():
        if _VARIANT and not hasattr(L, name):
            continue  # a kernel variant library: the decode ABI only (gpk_kernels.hip + gpk_host.cpp)
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(rc):
    if rc != GPK_OK:
        L = lib()
        raise GpkError("gpk: %s (%d) %s" % (L.gpk_strerror(rc).decode(), rc, L.gpk_last_hip_error().decode()))
    return rc


class _Mem:
    __slots__ = ("__array_interface__",)


def host_view(ptr, count, dtype):
    """A numpy array of `count` elements of `dtype` over library-owned host
    memory at `ptr` (an int or ctypes pointer), without copying. Built from the
    array interface rather than np.ctypeslib.as_array: that creates a ctypes
    array type per distinct length, which ctypes caches for the life of the
    process (about 4.5 KB each), so callbacks that see batches of varying size
    grew the process without bound."""
    dt = np.dtype(dtype)
    if ptr is not None and not isinstance(ptr, int):  # a ctypes pointer or c_void_p
        ptr = ctypes.cast(ptr, ctypes.c_void_p).value
    m = _Mem()
    m.__array_interface__ = {"data": (int(ptr or 0), False), "shape": (int(count),), "version": 3,
                             "typestr": dt.str if dt.fields is None else "|V%d" % dt.itemsize}
    a = np.asarray(m)
    return a if dt.fields is None else a.view(dt)


_synth = None


def synth_lib():
    """libgpk_synth.so: synthetic benchmark batches (bench/test infrastructure)."""
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_PATH):
            raise ImportError("gopacket_amd: %s is not built" % SYNTH_PATH)
        _share_hip_runtime()
        S = ctypes.CDLL(SYNTH_PATH)
        S.gpk_synth_len.argtypes = [ctypes.c_int, ctypes.c_uint64]
        S.gpk_synth_len.restype = ctypes.c_uint32
        S.gpk_synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]
        S.gpk_synth_fill.restype = ctypes.c_uint32
        S.gpk_synth_batch_host.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]
        S.gpk_synth_batch_host.restype = ctypes.c_uint64
        S.gpk_synth_device.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        S.gpk_synth_device.restype = ctypes.c_int
        S.gpk_synth_bytes.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        S.gpk_synth_bytes.restype = ctypes.c_uint64
        S.gpk_synth_write_pcapng.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_int]
        S.gpk_synth_write_pcapng.restype = ctypes.c_uint64
        S.gpk_probe_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_void_p]
        S.gpk_probe_read.restype = ctypes.c_int
        S.gpk_probe_reread.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p]
        S.gpk_probe_reread.restype = ctypes.c_int
        S.gpk_probe_mixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        S.gpk_probe_mixed.restype = ctypes.c_int
        S.gpk_probe_reread_lds.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        S.gpk_probe_reread_lds.restype = ctypes.c_int
        S.gpk_probe_skeleton.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        S.gpk_probe_skeleton.restype = ctypes.c_int
        S.gpk_probe_skeleton_idx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int,
                                             ctypes.c_void_p, ctypes.c_void_p]
        S.gpk_probe_skeleton_idx.restype = ctypes.c_int
        S.gpk_probe_skeleton_storer.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                                ctypes.c_void_p]
        S.gpk_probe_skeleton_storer.restype = ctypes.c_int
        S.gpk_probe_malloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint64, ctypes.c_uint]
        S.gpk_probe_malloc.restype = ctypes.c_int
        S.gpk_probe_free.argtypes = [ctypes.c_void_p]
        S.gpk_probe_free.restype = ctypes.c_int
        S.gpk_probe_d2d.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        S.gpk_probe_d2d.restype = ctypes.c_int
        S.gpk_probe_hostwrite.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        S.gpk_probe_hostwrite.restype = ctypes.c_int
        S.gpk_probe_h2d_rate.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int]
        S.gpk_probe_h2d_rate.restype = ctypes.c_double
        S.gpk_synth_tpacket_v3.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.c_uint64, ctypes.c_int32, ctypes.c_uint32, ctypes.c_void_p]
        S.gpk_synth_tpacket_v3.restype = ctypes.c_uint64
        S.gpk_synth_tp_producer_start.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        S.gpk_synth_tp_producer_start.restype = ctypes.c_void_p
        S.gpk_synth_tp_producer_stop.argtypes = [ctypes.c_void_p]
        S.gpk_synth_tp_producer_stop.restype = ctypes.c_uint64
        _synth = S
    return _synth
