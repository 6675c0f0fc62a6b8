"""afpacket-shaped ring reader over the native walker (include/gpk_afpacket.h).

Mirrors the reference's afpacket package for the ingest side of the path
(SURVEY.md §8(f)2):

  NewTPacket(*opts) -> TPacket                afpacket/afpacket.go:261-294
  Opt* option types, Default* constants       afpacket/options.go:22-132
  parseOptions(*opts)                         options.go:160-211 (error texts)
  TPacket.ZeroCopyReadPacketData()            afpacket.go:335-367
  TPacket.ReadPacketData() / ReadPacketDataTo afpacket.go:438-460
  TPacket.Stats() / SocketStats()             afpacket.go:370-431
  TPacket.SetBPF / SetFanout / Close          afpacket.go:297-309,542-548,243-254
  TPacket.SetEBPF / SetPromiscuous            afpacket.go:312-314,552-564
  TPacket.WritePacketData / InitSocketStats   afpacket.go:567-570,378-399

plus what the reference has no counterpart for:

  AttachRing(buf, version, *opts)             the same reader over a ring in
                                              caller memory (tests, replays, bench)
  TPacket.ReadBatch(max)                      the batch form (in-place offsets)
  TPacket.Pump(ctx, parser, ...)              ring -> HBM -> decode loop
                                              (gpk_tpacket_pump)

Errors carry the reference's text: ErrTimeout ("packet poll timeout
expired"), ErrPoll ("packet poll failed"). An attached ring has no socket to
poll: where the reference would block, ZeroCopyReadPacketData raises
WouldBlock.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .pcapgo import CaptureInfo

TPacketVersionHighestAvailable, TPacketVersion1, TPacketVersion2, TPacketVersion3 = -1, 0, 1, 2
SocketRaw, SocketDgram = 3, 2
DefaultFrameSize = 4096
DefaultBlockSize = DefaultFrameSize * 128
DefaultNumBlocks = 128
DefaultBlockTimeout = 64 * 1000000  # ns
DefaultPollTimeout = -1 * 1000000   # ns: blocks forever


class OptFrameSize(int): pass  # noqa: E701
class OptBlockSize(int): pass  # noqa: E701
class OptNumBlocks(int): pass  # noqa: E701
class OptBlockTimeout(int): pass  # noqa: E701  (nanoseconds, a time.Duration)
class OptPollTimeout(int): pass  # noqa: E701  (nanoseconds)
class OptTPacketVersion(int): pass  # noqa: E701
class OptProtocol(int): pass  # noqa: E701
class OptSocketType(int): pass  # noqa: E701
class OptVNetHdrSize(int): pass  # noqa: E701
class OptInterface(str): pass  # noqa: E701


class OptAddVLANHeader(int):  # a bool in Go
    pass


class AfpacketError(Exception):
    def __init__(self, text, panic=False):
        super().__init__(text)
        self.text = text
        self.panic = panic


ErrTimeoutText = "packet poll timeout expired"
ErrPollText = "packet poll failed"


class WouldBlock(Exception):
    """The next header is still the kernel's (an attached ring: nothing to poll)."""


@dataclass
class AncillaryVLAN:  # afpacket.go:45-48
    VLAN: int


@dataclass
class Stats:  # afpacket.go:51-58
    Packets: int
    Polls: int


@dataclass
class SocketStats:
    packets: int
    drops: int

    def Packets(self):
        return self.packets

    def Drops(self):
        return self.drops


@dataclass
class SocketStatsV3(SocketStats):
    freezeQCount: int = 0

    def QueueFreezes(self):
        return self.freezeQCount


def parseOptions(*opts):
    """-> _lib.TpOpts, or AfpacketError with Go's text."""
    L = _lib.lib()
    o = _lib.TpOpts()
    L.gpk_tp_default_opts(ctypes.byref(o))
    for v in opts:
        if isinstance(v, OptFrameSize):
            o.frame_size = int(v)
        elif isinstance(v, OptBlockSize):
            o.block_size = int(v)
        elif isinstance(v, OptNumBlocks):
            o.num_blocks = int(v)
        elif isinstance(v, OptBlockTimeout):
            o.block_timeout_ns = int(v)
        elif isinstance(v, OptPollTimeout):
            o.poll_timeout_ns = int(v)
        elif isinstance(v, OptTPacketVersion):
            o.version = int(v)
        elif isinstance(v, OptProtocol):
            o.protocol = int(v) & 0xFFFF
        elif isinstance(v, OptInterface):
            o.iface = str(v).encode()
        elif isinstance(v, OptSocketType):
            o.socktype = int(v)
        elif isinstance(v, OptAddVLANHeader):
            o.add_vlan_header = 1 if v else 0
        elif isinstance(v, OptVNetHdrSize):
            o.vnet_hdr_size = int(v)
        else:
            raise AfpacketError("unknown type in options")
    err = ctypes.create_string_buffer(256)
    if L.gpk_tp_check_opts(ctypes.byref(o), err, 256) != _lib.GPK_OK:
        raise AfpacketError(err.value.decode())
    return o


class TPacket:
    def __init__(self, h, keep=None):
        self.h = ctypes.c_void_p(h)
        self._keep = keep  # ring memory of an attached reader
        L = _lib.lib()
        ring, nbytes, ver, fd = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int(), ctypes.c_int()
        L.gpk_tpacket_ring(self.h, ctypes.byref(ring), ctypes.byref(nbytes), ctypes.byref(ver), ctypes.byref(fd))
        self.ring_ptr, self.ring_bytes, self.version, self.fd = ring.value, nbytes.value, ver.value, fd.value
        self.ring = _lib.host_view(ring, self.ring_bytes, np.uint8)
        self._side = np.zeros(1 << 20, np.uint8)

    def _error(self):
        buf = ctypes.create_string_buffer(256)
        pan = ctypes.c_int()
        _lib.lib().gpk_tpacket_error(self.h, buf, 256, ctypes.byref(pan))
        return AfpacketError(buf.value.decode(errors="replace"), bool(pan.value))

    def ReadBatch(self, max_pkts=1 << 16, wait=None):
        """Up to max_pkts packets: (list of packet bytes, offsets, caplens, tp_info array, status).
        Offsets >= ring bytes point into this reader's side buffer (VLAN-inserted copies)."""
        wait = (self.fd >= 0) if wait is None else wait
        off = np.zeros(max_pkts, np.uint64)
        cap = np.zeros(max_pkts, np.uint32)
        ci = np.zeros(max_pkts, _lib.TPINFO_DTYPE)
        n, used = ctypes.c_uint64(), ctypes.c_uint64()
        st = _lib.lib().gpk_tpacket_index(self.h, 1 if wait else 0, off.ctypes.data, cap.ctypes.data, ci.ctypes.data,
                                          max_pkts, ctypes.byref(n), self._side.ctypes.data, len(self._side),
                                          ctypes.byref(used))
        if st < 0:
            _lib.check(st)
        k = n.value
        pk = [self._bytes(int(o), int(c)) for o, c in zip(off[:k], cap[:k])]
        return pk, off[:k], cap[:k], ci[:k], st

    def _bytes(self, o, c):
        if o >= self.ring_bytes:
            o -= self.ring_bytes
            return bytes(self._side[o:o + c])
        return bytes(self.ring[o:o + c])

    def ZeroCopyReadPacketData(self):
        pk, off, cap, ci, st = self.ReadBatch(1)
        if not pk:
            if st == _lib.TP_ERROR:
                raise self._error()
            raise WouldBlock()
        c = ci[0]
        anc = [AncillaryVLAN(int(c["vlan"]))] if c["vlan"] >= 0 else []
        return pk[0], CaptureInfo((int(c["ts_sec"]), int(c["ts_nsec"])), int(cap[0]), int(c["length"]),
                                  int(c["iface"]), anc)

    def ReadPacketData(self):
        return self.ZeroCopyReadPacketData()

    def ReadPacketDataTo(self, buf):
        d, ci = self.ZeroCopyReadPacketData()
        k = min(len(buf), len(d))
        buf[:k] = d[:k]
        ci.CaptureLength = k
        return ci

    def Stats(self):
        p, q = ctypes.c_int64(), ctypes.c_int64()
        _lib.lib().gpk_tpacket_stats(self.h, ctypes.byref(p), ctypes.byref(q))
        return Stats(p.value, q.value)

    def SocketStats(self):
        a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _lib.check(_lib.lib().gpk_tpacket_socket_stats(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        if self.version == TPacketVersion3:
            return SocketStats(0, 0), SocketStatsV3(a.value, b.value, c.value)
        return SocketStats(a.value, b.value), SocketStatsV3(0, 0, 0)

    def SetBPF(self, insns):
        """insns: sequence of (code, jt, jf, k) classic BPF instructions (bpf.RawInstruction)."""
        if len(insns) > 0xFFFF:
            raise AfpacketError("filter too large")
        arr = np.zeros(len(insns), np.dtype([("code", "<u2"), ("jt", "u1"), ("jf", "u1"), ("k", "<u4")]))
        for i, (c, jt, jf, k) in enumerate(insns):
            arr[i] = (c, jt, jf, k)
        _lib.check(_lib.lib().gpk_tpacket_set_bpf(self.h, arr.ctypes.data if len(arr) else None, len(arr)))

    def SetFanout(self, t, id_):
        _lib.check(_lib.lib().gpk_tpacket_set_fanout(self.h, int(t), int(id_)))

    def SetEBPF(self, prog_fd):  # afpacket.go:312-314
        _lib.check(_lib.lib().gpk_tpacket_set_ebpf(self.h, int(prog_fd)))

    def SetPromiscuous(self, on):  # afpacket.go:552-564
        _lib.check(_lib.lib().gpk_tpacket_set_promiscuous(self.h, 1 if on else 0))

    def WritePacketData(self, pkt):  # afpacket.go:567-570
        b = bytes(pkt)
        _lib.check(_lib.lib().gpk_tpacket_write(self.h, b, len(b)))

    def InitSocketStats(self):  # afpacket.go:378-399
        _lib.check(_lib.lib().gpk_tpacket_init_socket_stats(self.h))

    def Pump(self, ctx, parser, batch_pkts=0, max_packets=0, wait=False, inflight=0, collect=True, on_batch=None,
             fields=False, packets=False):
        """gpk_tpacket_pump: drain the ring through HBM and the decoder. Returns
        (results-or-None, stats dict); results as Context.replay_file's, with
        ci of TPINFO_DTYPE. fields=True: every launch is the fused decode +
        layer fields (gpk_tp_pump_opts.fields_cb); results gain "fields" and
        on_batch a last argument, as in replay_file. packets=True (collect=False
        only): on_batch also gets, last, (pointers, caplens): packet i's bytes
        are ctypes.string_at(pointers[i], caplens[i]) (a ring frame or its VLAN
        copy, valid during the call); ring headers go back to the kernel once
        their batch was delivered. A callback that raises ends the pump at
        once (gpk_stop) and the exception is raised from here; ctx.stop() from
        a callback or another thread ends it too (stats["stopped"])."""
        if packets and collect:
            raise ValueError("packets=True hands out views of the ring: use collect=False and on_batch")
        parts = []
        got_fields = []
        got_packets = []

        raised = []  # an exception inside a ctypes callback would be printed and dropped: kept for after the call

        def guarded(f):  # every callback: the first exception is kept, ends the pump, and is re-raised after it
            def g(*args):
                if not raised:
                    try:
                        f(*args)
                    except BaseException as e:  # noqa: B902 (re-raised below, after the C call returns)
                        raised.append(e)
                        _lib.lib().gpk_stop(ctx.h)  # no further callback: the pump drains and returns
            return g

        @guarded
        def pcb(user, first, n, data, cap):
            if n:
                got_packets[:] = [(first, n, (_lib.host_view(data, n, np.uint64), _lib.host_view(cap, n, np.uint32)))]

        @guarded
        def fcb(user, first, n, f):
            got_fields[:] = [(first, n, _lib.host_view(f, n, _lib.FIELDS_DTYPE) if n else np.zeros(0, _lib.FIELDS_DTYPE))]

        def cb(*args):
            guarded(_cb)(*args)

        def _cb(user, first, n, rec, err, fl, ci, cap):
            if not n:
                return
            views = (_lib.host_view(rec, n, _lib.RECORD_DTYPE), _lib.host_view(err, 2 * n, np.uint32),
                     _lib.host_view(fl, 3 * n, np.uint64), _lib.host_view(ci, n, _lib.TPINFO_DTYPE),
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

        c_cb = _lib.PUMP_CB(cb)
        c_fcb = _lib.PUMP_FIELDS_CB(fcb) if fields else _lib.PUMP_FIELDS_CB()
        c_pcb = _lib.PUMP_PACKETS_CB(pcb) if packets else _lib.PUMP_PACKETS_CB()
        o = _lib.PumpOpts(batch_pkts, max_packets, 1 if wait else 0, inflight, c_fcb, c_pcb)
        st = _lib.PumpStats()
        rc = _lib.lib().gpk_tpacket_pump(ctx.h, parser.h, self.h, ctypes.byref(o), c_cb, None, ctypes.byref(st))
        if raised:
            raise raised[0]
        if rc not in (_lib.GPK_OK, _lib.GPK_STOPPED):
            raise _lib.GpkError("gpk_tpacket_pump: %d %s %s" % (rc, st.error.decode(errors="replace"),
                                                                _lib.lib().gpk_last_hip_error().decode()))
        stats = {k: getattr(st, k) for k, _ in _lib.PumpStats._fields_}
        stats["error"] = st.error.decode(errors="replace")
        stats["kernel"] = st.kernel.decode(errors="replace")
        stats["stopped"] = rc == _lib.GPK_STOPPED
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
                           flows=np.zeros(0, np.uint64), ci=np.zeros(0, _lib.TPINFO_DTYPE),
                           caplens=np.zeros(0, np.uint32))
                if fields:
                    res["fields"] = np.zeros(0, _lib.FIELDS_DTYPE)
        return res, stats

    def Close(self):
        if self.h:
            _lib.lib().gpk_tpacket_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.Close()
        except Exception:
            pass


def NewTPacket(*opts):
    o = parseOptions(*opts)
    h = ctypes.c_void_p()
    err = ctypes.create_string_buffer(256)
    rc = _lib.lib().gpk_tpacket_new(ctypes.byref(h), ctypes.byref(o), err, 256)
    if rc != _lib.GPK_OK:
        raise AfpacketError(err.value.decode(errors="replace"))
    return TPacket(h.value)


def AttachRing(buf, version, *opts):
    """A reader over buf (numpy uint8 array / bytearray, kept alive by the
    reader) laid out as the kernel's ring of `version` with opts' geometry."""
    o = parseOptions(*opts)
    arr = buf if isinstance(buf, np.ndarray) else np.frombuffer(buf, np.uint8)
    h = ctypes.c_void_p()
    _lib.check(_lib.lib().gpk_tpacket_attach(ctypes.byref(h), arr.ctypes.data, arr.nbytes, int(version),
                                             ctypes.byref(o)))
    return TPacket(h.value, keep=arr)
