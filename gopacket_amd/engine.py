"""Thin object layer over the C ABI: parser configuration, device context and
batch decode calls (host-memory and device-resident). The gopacket-shaped API
(DecodingLayerParser, layers.*) in parser.py / layers.py is built on this.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib

DECODER_KINDS = {
    "Ethernet": _lib.DEC_ETHERNET, "Dot1Q": _lib.DEC_DOT1Q, "IPv4": _lib.DEC_IPV4, "IPv6": _lib.DEC_IPV6,
    "IPv6ExtensionSkipper": _lib.DEC_IPV6_EXT, "TCP": _lib.DEC_TCP, "UDP": _lib.DEC_UDP,
    "Payload": _lib.DEC_PAYLOAD, "Fragment": _lib.DEC_FRAGMENT,
}


class ParserConfig:
    """gpk_parser: container + options + next-layer tables (parser.go:182-241)."""

    def __init__(self, first, decoder_kinds=(), ignore_panic=False, ignore_unsupported=False,
                 outputs=_lib.OUT_ALL):
        h = ctypes.c_void_p()
        check(lib().gpk_parser_create(ctypes.byref(h), int(first)))
        self.h = h
        self.first = int(first)
        for k in decoder_kinds:
            self.add_decoder(k)
        self.set_options(ignore_panic, ignore_unsupported)
        self.set_outputs(outputs)

    def add_decoder(self, kind):
        check(lib().gpk_parser_add_decoder(self.h, int(kind)))

    def set_options(self, ignore_panic, ignore_unsupported):
        self.ignore_panic = bool(ignore_panic)
        self.ignore_unsupported = bool(ignore_unsupported)
        check(lib().gpk_parser_set_options(self.h, int(self.ignore_panic), int(self.ignore_unsupported)))

    def set_outputs(self, outputs):
        self.outputs = int(outputs)
        check(lib().gpk_parser_set_outputs(self.h, self.outputs))

    def decoder_for(self, layer_type):
        return lib().gpk_parser_decoder_for(self.h, int(layer_type))

    def set_ethertype(self, v, lt):
        check(lib().gpk_parser_set_ethertype(self.h, int(v), int(lt)))

    def set_ipprotocol(self, v, lt):
        check(lib().gpk_parser_set_ipprotocol(self.h, int(v), int(lt)))

    def set_tcp_port(self, v, lt):
        check(lib().gpk_parser_set_tcp_port(self.h, int(v), int(lt)))

    def set_udp_port(self, v, lt):
        check(lib().gpk_parser_set_udp_port(self.h, int(v), int(lt)))

    def __del__(self):
        h = getattr(self, "h", None)
        L = getattr(_lib, "_lib", None) if _lib is not None else None  # module globals are None at exit
        if h and L is not None:
            L.gpk_parser_destroy(h)
            self.h = None


class Context:
    """gpk_ctx: one GPU."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        check(lib().gpk_ctx_create(ctypes.byref(h), int(device)))
        self.h = h
        self.device = device

    def __del__(self):
        h = getattr(self, "h", None)
        L = getattr(_lib, "_lib", None) if _lib is not None else None  # module globals are None at exit
        if h and L is not None:
            L.gpk_ctx_destroy(h)
            self.h = None

    def set_table_mode(self, mode):
        """_lib.TABLES_AUTO (compact LDS tables when they fit) or TABLES_GLOBAL."""
        check(lib().gpk_ctx_set_table_mode(self.h, int(mode)))

    def stop(self):
        """gpk_stop: end the replay_file / Pump.run calls running on this
        context (a Go caller's break out of its ReadPacketData loop); callable
        from their callbacks or from another thread."""
        check(lib().gpk_stop(self.h))

    def decode_host(self, parser, data, offsets, caplens, layouts=False, fields=False):
        """Host batch in, host results out (copies HtoD, decodes, copies DtoH).
        fields=True: gpk_decode_batch_host_fields, the results gain "fields"
        (FIELDS_DTYPE per packet; the fused launch, or with layouts the decode
        then the extraction)."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        caplens = np.ascontiguousarray(caplens, dtype=np.uint32)
        n = len(offsets)
        if n and np.any(offsets.astype(np.uint64) + caplens.astype(np.uint64) > len(data)):
            raise ValueError("packet range outside the data buffer")
        rec = np.zeros(n, _lib.RECORD_DTYPE)
        err = np.zeros(2 * n, np.uint32)
        flows = np.zeros(3 * n, np.uint64)
        lay = np.zeros(n, _lib.LAYOUT_DTYPE) if layouts else None
        b = _lib.Batch(data.ctypes.data, offsets.ctypes.data, caplens.ctypes.data, n, len(data))
        r = _lib.Results(rec.ctypes.data, err.ctypes.data, flows.ctypes.data,
                         lay.ctypes.data if layouts else None)
        if fields:
            fld = np.zeros(n, _lib.FIELDS_DTYPE)
            check(lib().gpk_decode_batch_host_fields(self.h, parser.h, ctypes.byref(b), ctypes.byref(r),
                                                     fld.ctypes.data if n else None))
            return dict(records=rec, err_args=err, flows=flows, layouts=lay, fields=fld)
        check(lib().gpk_decode_batch_host(self.h, parser.h, ctypes.byref(b), ctypes.byref(r)))
        return dict(records=rec, err_args=err, flows=flows, layouts=lay)

    def decode_device(self, parser, data, offsets, caplens, records, err_args=None, flows=None, layouts=None,
                      stream=None):
        """Device-resident decode: every argument is a torch CUDA tensor (or an
        object with data_ptr()); enqueued on `stream` (torch stream or raw handle)."""
        n = offsets.numel()
        b = _lib.Batch(data.data_ptr(), offsets.data_ptr(), caplens.data_ptr(), n, data.numel())
        r = _lib.Results(records.data_ptr(), err_args.data_ptr() if err_args is not None else None,
                         flows.data_ptr() if flows is not None else None,
                         layouts.data_ptr() if layouts is not None else None)
        check(lib().gpk_decode_batch(self.h, parser.h, ctypes.byref(b), ctypes.byref(r), _stream_ptr(stream)))

    def decode_device_narrow(self, parser, data, offsets, caplens, records8, wide, err_args=None, flows=None,
                             stream=None):
        """gpk_decode_batch_narrow: decode_device with the 8-byte record
        (records8: 8 bytes per packet, RECORD8_DTYPE) and the side array of full
        records (wide: 16 bytes per packet, written only where a record8 has
        ST8_WIDE). Device tensors; enqueued on `stream`."""
        n = offsets.numel()
        if records8.numel() * records8.element_size() < 8 * n or wide.numel() * wide.element_size() < 16 * n:
            raise ValueError("records8 needs 8 and wide 16 bytes per packet")
        b = _lib.Batch(data.data_ptr(), offsets.data_ptr(), caplens.data_ptr(), n, data.numel())
        r = _lib.Results8(records8.data_ptr(), wide.data_ptr(), err_args.data_ptr() if err_args is not None else None,
                          flows.data_ptr() if flows is not None else None)
        check(lib().gpk_decode_batch_narrow(self.h, parser.h, ctypes.byref(b), ctypes.byref(r), _stream_ptr(stream)))

    def extract_fields(self, data, offsets, caplens, layouts, fields, stream=None):
        """gpk_extract_fields: the layer fields (include/gpk.h gpk_fields, 128
        bytes per packet; FIELDS_DTYPE) of a device batch from the layouts a
        decode_device of it wrote. Device tensors; enqueued on `stream`."""
        n = offsets.numel()
        if fields.numel() * fields.element_size() < 128 * n or layouts.numel() * layouts.element_size() < 64 * n:
            raise ValueError("fields needs 128 bytes and layouts 64 bytes per packet")
        b = _lib.Batch(data.data_ptr(), offsets.data_ptr(), caplens.data_ptr(), n, data.numel())
        check(lib().gpk_extract_fields(ctypes.byref(b), layouts.data_ptr(), fields.data_ptr(), _stream_ptr(stream)))

    def decode_device_fields(self, parser, data, offsets, caplens, records, err_args, flows, fields, layouts=None,
                             stream=None):
        """gpk_decode_batch_fields: decode_device plus the layer fields of every
        packet (fields: 128 bytes per packet, FIELDS_DTYPE) in one launch
        (layouts=None), or decode with layouts + extract_fields. Device tensors."""
        n = offsets.numel()
        if fields.numel() * fields.element_size() < 128 * n:
            raise ValueError("fields needs 128 bytes per packet")
        b = _lib.Batch(data.data_ptr(), offsets.data_ptr(), caplens.data_ptr(), n, data.numel())
        r = _lib.Results(records.data_ptr(), err_args.data_ptr() if err_args is not None else None,
                         flows.data_ptr() if flows is not None else None,
                         layouts.data_ptr() if layouts is not None else None)
        check(lib().gpk_decode_batch_fields(self.h, parser.h, ctypes.byref(b), ctypes.byref(r), fields.data_ptr(),
                                            _stream_ptr(stream)))

    def decode_host_fields(self, parser, data, offsets, caplens, layouts=True):
        """decode_host plus the layer fields of every packet, both computed on
        the device (gpk_decode_batch_host_fields; host arrays in and out).
        layouts=True: the decode with layouts, then extract_fields from them
        (two launches); False: the fused decode + fields launch, no layouts
        returned. Returns (results, fields)."""
        r = self.decode_host(parser, data, offsets, caplens, layouts=layouts, fields=True)
        return r, r.pop("fields")

    def kernel_name(self, parser, data, offsets, caplens, layouts=False):
        """The decode kernel specialisation decode_device (torch tensors) or
        decode_host (numpy arrays) launches for this parser and batch
        (gpk_decode_kernel_name): the name rocprofv3 lists. layouts=
        _lib.NAME_FIELDS: the fused decode + fields launch."""
        b = _batch_of(data, offsets, caplens)
        buf = ctypes.create_string_buffer(256)
        n = lib().gpk_decode_kernel_name(self.h, parser.h, ctypes.byref(b), int(layouts), buf, 256)
        if n < 0:
            raise _lib.GpkError("gpk_decode_kernel_name: %d" % n)
        return buf.value.decode()

    def occupancy(self, parser, data, offsets, caplens, layouts=False):
        """Blocks of that kernel resident per CU with this parser's LDS table
        blob (gpk_decode_occupancy)."""
        b = _batch_of(data, offsets, caplens)
        out = ctypes.c_int()
        check(lib().gpk_decode_occupancy(self.h, parser.h, ctypes.byref(b), int(layouts), ctypes.byref(out)))
        return out.value

    def replay_file(self, parser, path, fmt=0, ng_flags=0, slot_bytes=0, slots=0, batch_pkts=0, read_threads=0,
                    collect=True, on_batch=None, fields=False, packets=False, byte_range=None):
        """gpk_replay_file: the whole capture through HBM (BASELINE config C5).
        collect=True gathers every result (records, err_args, flows SoA, ci,
        caplens) in packet order; on_batch(first, n, records, err_args, flows,
        ci, caplens) sees each launch's numpy views instead (valid during the
        call). fields=True: every launch is the fused decode + layer fields
        (gpk_replay_opts.fields_cb): the results gain "fields" (FIELDS_DTYPE
        per packet), and on_batch a last argument, the launch's fields.
        packets=True (collect=False only): on_batch also gets, last, the
        launch's packets as (data, offsets, caplens): packet i is
        data[offsets[i]:offsets[i] + caplens[i]], a view of the staging buffer
        the file was read into (gpk_replay_opts.packets_cb; no copy, valid
        during the call). byte_range=(begin, end): one caller's share of the
        file (gpk_replay_file_range; end 0 = the file's end); the stats then
        carry "range" (header_end, sync_begin, sync_end, clean, state_changed).
        A callback that raises ends the call at once (gpk_stop: no further
        callback), and the exception is raised from here; a callback, or another
        thread, may also end it with ctx.stop(): stats["stopped"] is then True
        and the results hold the packets delivered before it.
        Returns (results-or-None, stats dict)."""
        if packets and collect:
            raise ValueError("packets=True hands out views of the staging buffers: use collect=False and on_batch")
        parts = []
        got_packets = []

        raised = []  # an exception inside a ctypes callback would be printed and dropped: kept for after the call

        def guarded(f):  # every callback: the first exception is kept, ends the call, and is re-raised after it
            def g(*args):
                if not raised:
                    try:
                        f(*args)
                    except BaseException as e:  # noqa: B902 (re-raised below, after the C call returns)
                        raised.append(e)
                        lib().gpk_stop(self.h)  # no further callback: the call drains and returns
            return g

        @guarded
        def pcb(user, first, n, base, nbytes, off, cap):
            if not n:
                return
            o = _lib.host_view(off, n, np.uint64)
            c = _lib.host_view(cap, n, np.uint32)
            data = _lib.host_view(base, max(nbytes, 1), np.uint8)
            got_packets[:] = [(first, n, (data, o, c))]
        got_fields = []  # the current launch's fields (fields_cb runs right before cb)

        @guarded
        def fcb(user, first, n, f):
            got_fields[:] = [(first, n, _lib.host_view(f, n, _lib.FIELDS_DTYPE) if n else np.zeros(0, _lib.FIELDS_DTYPE))]

        def cb(*args):
            guarded(_cb)(*args)

        def _cb(user, first, n, rec, err, fl, ci, cap):
            if not n:
                return
            views = (_lib.host_view(rec, n, _lib.RECORD_DTYPE), _lib.host_view(err, 2 * n, np.uint32),
                     _lib.host_view(fl, 3 * n, np.uint64), _lib.host_view(ci, n, _lib.CAPINFO_DTYPE),
                     _lib.host_view(cap, n, np.uint32))
            if fields:  # the library calls fields_cb for the same packets right before this
                if not got_fields or got_fields[0][:2] != (first, n):
                    raise RuntimeError("no layer fields delivered for packets %d..%d" % (first, first + n))
                views = views + (got_fields.pop()[2],)
            if packets:
                if not got_packets or got_packets[0][:2] != (first, n):
                    raise RuntimeError("no packets delivered for packets %d..%d" % (first, first + n))
                views = views + (got_packets.pop()[2],)
            if on_batch is not None:
                on_batch(first, n, *views)
            if collect:
                parts.append(tuple(v.copy() for v in views))

        c_cb = _lib.REPLAY_CB(cb)
        c_fcb = _lib.REPLAY_FIELDS_CB(fcb) if fields else _lib.REPLAY_FIELDS_CB()
        c_pcb = _lib.REPLAY_PACKETS_CB(pcb) if packets else _lib.REPLAY_PACKETS_CB()
        o = _lib.ReplayOpts(fmt, ng_flags, slot_bytes, slots, batch_pkts, read_threads, c_fcb, c_pcb)
        st = _lib.ReplayStats()
        cpath = path.encode() if isinstance(path, str) else path
        rg = None
        if byte_range is None:
            rc = lib().gpk_replay_file(self.h, parser.h, cpath, ctypes.byref(o), c_cb, None, ctypes.byref(st))
        else:
            rg = _lib.ReplayRange(int(byte_range[0]), int(byte_range[1]))
            rc = lib().gpk_replay_file_range(self.h, parser.h, cpath, ctypes.byref(rg), ctypes.byref(o), c_cb, None,
                                             ctypes.byref(st))
        if raised:
            raise raised[0]
        if rc not in (_lib.GPK_OK, _lib.GPK_STOPPED):
            err = _lib.GpkError("gpk_replay_file: %d %s %s" % (rc, st.error.decode(errors="replace"),
                                                              lib().gpk_last_hip_error().decode()))
            if rg is not None:  # where the range was cut, for the caller's redo (shard.replay_file_sharded)
                err.range = {k: int(getattr(rg, k)) for k, _ in _lib.ReplayRange._fields_}
            raise err
        stats = {k: getattr(st, k) for k, _ in _lib.ReplayStats._fields_}
        stats["error"] = st.error.decode(errors="replace")
        stats["kernel"] = st.kernel.decode(errors="replace")
        stats["stopped"] = rc == _lib.GPK_STOPPED
        if rg is not None:
            stats["range"] = {k: int(getattr(rg, k)) for k, _ in _lib.ReplayRange._fields_}
        res = None
        if collect:
            if parts:
                fl = np.concatenate([p[2].reshape(3, -1) for p in parts], axis=1).reshape(-1)
                res = dict(records=np.concatenate([p[0] for p in parts]), err_args=np.concatenate([p[1] for p in parts]),
                           flows=fl, ci=np.concatenate([p[3] for p in parts]), caplens=np.concatenate([p[4] for p in parts]))
                if fields:
                    res["fields"] = np.concatenate([p[5] for p in parts])
            else:
                res = dict(records=np.zeros(0, _lib.RECORD_DTYPE), err_args=np.zeros(0, np.uint32),
                           flows=np.zeros(0, np.uint64), ci=np.zeros(0, _lib.CAPINFO_DTYPE),
                           caplens=np.zeros(0, np.uint32))
                if fields:
                    res["fields"] = np.zeros(0, _lib.FIELDS_DTYPE)
        return res, stats

    def decoded_list_host(self, parser, pkt, cap=65536):
        out = (ctypes.c_int64 * cap)()
        n = ctypes.c_uint32()
        pkt = bytes(pkt)
        check(lib().gpk_decoded_list_host(self.h, parser.h, pkt, len(pkt), out, cap, ctypes.byref(n)))
        return [out[i] for i in range(min(n.value, cap))]


def _batch_of(data, offsets, caplens):
    """gpk_batch over torch tensors or numpy arrays (the pointers are only
    described, never dereferenced, by the name / occupancy queries)."""
    if isinstance(data, np.ndarray):
        return _lib.Batch(data.ctypes.data, offsets.ctypes.data, caplens.ctypes.data, len(offsets), data.nbytes)
    return _lib.Batch(data.data_ptr(), offsets.data_ptr(), caplens.data_ptr(), offsets.numel(), data.numel())


def _stream_ptr(stream):
    """A raw hipStream_t from a torch stream, an int handle or None."""
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def format_error(code, a0=0, a1=0):
    buf = ctypes.create_string_buffer(512)
    lib().gpk_format_error(int(code), int(a0) & 0xFFFFFFFF, int(a1) & 0xFFFFFFFF, buf, 512)
    return buf.value.decode()


def layer_type_name(lt):
    buf = ctypes.create_string_buffer(128)
    lib().gpk_layer_type_name(int(lt), buf, 128)
    return buf.value.decode()


CODE_TO_LAYER_TYPE = (0, 17, 15, 20, 21, 46, 47, 48, 49, 44, 45, 2, 3)


def decode_codes(layers_word, n):
    """The inline decoded list of a gpk_record (first min(n,16) entries)."""
    w = int(layers_word)
    return [CODE_TO_LAYER_TYPE[(w >> (4 * k)) & 15] for k in range(min(n, _lib.MAX_INLINE_LAYERS))]
