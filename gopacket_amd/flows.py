"""Flow-keyed grouping of a decoded batch on the device (include/gpk_flows.h,
SURVEY.md §8(f)3): the keying the reference's flow consumers do per packet
with a Go map, for a whole batch in HBM.

  Grouper(max_packets).group(...)          gpk_group_batch
  kind CONNECTION                          tcpassembly key{netFlow, TransportFlow()}
                                           (tcpassembly/assembly.go:292,525-545)
  kind DEFRAG                              ip4defrag ipv4{NetworkFlow(), Id}
                                           (ip4defrag/defrag.go:85-105,328-341)
  kind NET_BUCKET                          int(NetworkFlow().FastHash()) & (buckets-1)
                                           (doc.go:219-225)

Groups come in order of first appearance; packets inside a group in batch
order. group_of[i] < 0 says why packet i has no key (GROUP_* codes).
"""
import ctypes

from . import _lib

CONNECTION, DEFRAG, NET_BUCKET = _lib.GROUP_CONNECTION, _lib.GROUP_DEFRAG, _lib.GROUP_NET_BUCKET
NONE, USELESS, FRAG_TOO_SMALL, FRAG_OFFSET, FRAG_OVERRUN, UNKNOWN = (
    _lib.GROUP_NONE, _lib.GROUP_USELESS, _lib.GROUP_FRAG_TOO_SMALL, _lib.GROUP_FRAG_OFFSET,
    _lib.GROUP_FRAG_OVERRUN, _lib.GROUP_UNKNOWN)


class Grouper:
    def __init__(self, max_packets, device=0):
        self.h = ctypes.c_void_p()
        _lib.check(_lib.lib().gpk_grouper_create(ctypes.byref(self.h), device, int(max_packets)))
        self.max_packets = int(max_packets)

    def group(self, data, offsets, caplens, records, layouts=None, flows=None, kind=CONNECTION, buckets=8,
              out=None, stream=None):
        """Device tensors in (torch, as gpk_decode_batch takes them); returns
        dict(group_of, perm, start, first, counts) of device tensors (or fills `out`)."""
        import torch
        n = offsets.numel()
        dev = offsets.device
        if out is None:
            out = dict(group_of=torch.empty(n, dtype=torch.int32, device=dev),
                       perm=torch.empty(n, dtype=torch.int32, device=dev),
                       start=torch.empty(n + 1, dtype=torch.int32, device=dev),
                       first=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                       counts=torch.zeros(2, dtype=torch.int32, device=dev))
        b = _lib.Batch(data.data_ptr(), offsets.data_ptr(), caplens.data_ptr(), n, data.numel())
        r = _lib.Results(records.data_ptr(), None, flows.data_ptr() if flows is not None else None,
                         layouts.data_ptr() if layouts is not None else None)
        g = _lib.Groups(out["group_of"].data_ptr(), out["perm"].data_ptr(), out["start"].data_ptr(),
                        out["first"].data_ptr(), out["counts"].data_ptr())
        sp = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
        _lib.check(_lib.lib().gpk_group_batch(self.h, ctypes.byref(b), ctypes.byref(r), int(kind), int(buckets),
                                              ctypes.byref(g), sp))
        return out

    def decode_group(self, ctx, parser, data, offsets, caplens, records, err_args=None, flows=None, kind=CONNECTION,
                     out=None, stream=None):
        """gpk_decode_group_batch: decode (records/err_args/flows as
        Context.decode_device, no layouts) and group by `kind` (CONNECTION or
        DEFRAG) with the key derived inside the decode kernel."""
        import torch
        n = offsets.numel()
        dev = offsets.device
        if out is None:
            out = dict(group_of=torch.empty(n, dtype=torch.int32, device=dev),
                       perm=torch.empty(n, dtype=torch.int32, device=dev),
                       start=torch.empty(n + 1, dtype=torch.int32, device=dev),
                       first=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                       counts=torch.zeros(2, dtype=torch.int32, device=dev))
        b = _lib.Batch(data.data_ptr(), offsets.data_ptr(), caplens.data_ptr(), n, data.numel())
        r = _lib.Results(records.data_ptr(), err_args.data_ptr() if err_args is not None else None,
                         flows.data_ptr() if flows is not None else None, None)
        g = _lib.Groups(out["group_of"].data_ptr(), out["perm"].data_ptr(), out["start"].data_ptr(),
                        out["first"].data_ptr(), out["counts"].data_ptr())
        sp = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
        _lib.check(_lib.lib().gpk_decode_group_batch(ctx.h, parser.h, ctypes.byref(b), ctypes.byref(r), self.h,
                                                     int(kind), ctypes.byref(g), sp))
        return out

    @staticmethod
    def to_lists(out):
        """Host view: (groups: list of packet-index lists in group order, group_of list)."""
        counts = out["counts"].cpu().tolist()
        G, K = counts[0], counts[1]
        perm = out["perm"][:K].cpu().tolist()
        start = out["start"][:G + 1].cpu().tolist()
        return [perm[start[g]:start[g + 1]] for g in range(G)], out["group_of"].cpu().tolist()

    def close(self):
        if self.h:
            _lib.lib().gpk_grouper_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pack_batch(data, offsets, caplens, order, total_bytes=None, stream=None):
    """gpk_pack_batch: the packets `order` (device int32 tensor) of a device
    batch, made dense in that order. Returns (data, offsets, caplens) tensors."""
    import torch
    m = order.numel()
    dev = order.device
    if total_bytes is None:
        total_bytes = int(caplens.index_select(0, order.long()).sum(dtype=torch.int64).item()) if m else 0
    out_d = torch.empty(total_bytes + 16, dtype=torch.uint8, device=dev)
    out_o = torch.empty(max(m, 1), dtype=torch.int64, device=dev)
    out_c = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
    b = _lib.Batch(data.data_ptr(), offsets.data_ptr(), caplens.data_ptr(), offsets.numel(), data.numel())
    sp = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
    _lib.check(_lib.lib().gpk_pack_batch(ctypes.byref(b), order.data_ptr() if m else None, m, out_d.data_ptr(),
                                         out_o.data_ptr(), out_c.data_ptr(), sp))
    return out_d, out_o[:m], out_c[:m]
