"""Multi-GPU sharding of a packet batch.

Every packet decodes independently (DecodeLayers resets its state per packet,
parser.go:304, layers_decoder.go:20), so a batch splits into contiguous
per-GPU ranges with no collective on the data path; results are disjoint
index ranges that concatenate. One process per GPU (torch.distributed),
each decoding its range on its own HIP stream.

The one step with a real exchange is flow affinity across GPUs: the
reference's sharding idiom (doc.go:219-225, channels[FastHash() & 7]) at node
scale, where every rank must end up with all packets of its flows (both
directions). exchange_packets does that with three all-to-alls (counts,
capture lengths, packet bytes); over RCCL they run on xGMI.
"""
import numpy as np


def weak_range(rank, n_per_rank):
    """Weak scaling (bench.py): rank r owns packets [r*n, (r+1)*n)."""
    return rank * n_per_rank, n_per_rank


def byte_balanced_bounds(caplens, world):
    """Strong scaling of one batch: split at sum(caplen)*k/world so every GPU
    reads about the same number of bytes (IMIX batches are size-skewed).
    Returns world+1 packet indices."""
    caplens = np.asarray(caplens, dtype=np.uint64)
    csum = np.concatenate([[0], np.cumsum(caplens, dtype=np.uint64)])
    total = int(csum[-1])
    cuts = [0]
    for k in range(1, world):
        cuts.append(int(np.searchsorted(csum, total * k // world, side="left")))
    cuts.append(len(caplens))
    return cuts


def max_over_ranks(x, world, device=None):
    """Job time = the slowest rank's time (bench.py contract). At world size 1
    without a process group it is x itself."""
    import torch
    import torch.distributed as dist
    if world == 1 and not dist.is_initialized():
        return x
    if dist.get_backend() == "gloo":
        device = None  # gloo reduces host tensors
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def exchange_packets(data, offsets, caplens, dest, world, group=None, pack=None):
    """All-to-all of whole packets: packet i goes to rank dest[i] (dest[i] < 0:
    dropped). Every rank calls it with its own batch (torch tensors on its
    device for RCCL, CPU tensors for gloo). Returns (data, offsets, caplens,
    src_rank, src_index) of the packets this rank receives, ordered by source
    rank, then by the source's batch order.

    pack(data, offsets, caplens, order) -> (dense bytes, offsets, caplens):
    gopacket_amd.flows.pack_batch (the HIP kernel) by default; a test on
    CPU tensors passes its own."""
    import torch
    import torch.distributed as dist
    if pack is None:
        from .flows import pack_batch as pack
    dev = offsets.device
    dest = dest.to(torch.int64)
    keep = dest >= 0
    key = torch.where(keep, dest, torch.full_like(dest, world))
    _, order = torch.sort(key, stable=True)
    n_keep = int(keep.sum().item())
    order = order[:n_keep].to(torch.int32)
    send_pkts = torch.bincount(dest[keep], minlength=world).to(torch.int64)
    pdata, _, pcap = pack(data, offsets, caplens, order)
    pcap64 = pcap.to(torch.int64)
    bounds = torch.cumsum(send_pkts, 0)
    csum = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), torch.cumsum(pcap64, 0)])
    send_bytes = csum[bounds] - csum[bounds - send_pkts]
    recv_pkts = torch.empty_like(send_pkts)
    recv_bytes = torch.empty_like(send_bytes)
    dist.all_to_all_single(recv_pkts, send_pkts, group=group)
    dist.all_to_all_single(recv_bytes, send_bytes, group=group)
    sp, rp = send_pkts.tolist(), recv_pkts.tolist()
    sb, rb = send_bytes.tolist(), recv_bytes.tolist()
    r_cap = torch.empty(sum(rp), dtype=torch.int32, device=dev)
    r_idx = torch.empty(sum(rp), dtype=torch.int32, device=dev)
    r_data = torch.empty(sum(rb) + 16, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(r_cap, pcap.contiguous(), output_split_sizes=rp, input_split_sizes=sp, group=group)
    dist.all_to_all_single(r_idx, order.contiguous(), output_split_sizes=rp, input_split_sizes=sp, group=group)
    dist.all_to_all_single(r_data[:sum(rb)], pdata[:sum(sb)].contiguous(), output_split_sizes=rb,
                           input_split_sizes=sb, group=group)
    r_off = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev),
                       torch.cumsum(r_cap.to(torch.int64), 0)[:-1]]) if len(r_cap) else r_cap.to(torch.int64)
    src = torch.repeat_interleave(torch.arange(world, device=dev), torch.tensor(rp, device=dev))
    return r_data, r_off, r_cap, src, r_idx


# ---- one capture file replayed by N ranks (C5 at N GPUs) ---------------------
def file_range(size, rank, world):
    """Rank r's cut of a file of `size` bytes: [size*r/N, size*(r+1)/N), the
    last one to the end (0). gpk_replay_file_range moves each cut to the next
    block start (include/gpk_capture.h)."""
    begin = size * rank // world
    end = 0 if rank == world - 1 else size * (rank + 1) // world
    return begin, end


def first_inexact(ranges):
    """The first rank whose share breaks the concatenation (None: exact).
    ranges: every rank's gpk_replay_range outputs in rank order. Rank k < N-1
    must have met io.EOF exactly at its sync_end (clean) with no section or
    interface block inside its range (state_changed); the last rank's end is
    the file's, whatever it holds (ngread.go:494-718)."""
    for k, r in enumerate(ranges[:-1]):
        if not r["clean"] or r["state_changed"]:
            return k
    return None


def replay_file_sharded(ctx, parser, path, rank, world, gather=None, **kw):
    """Rank `rank` of `world` replays its byte range of the pcapng file at
    `path` (Context.replay_file(byte_range=...), no data exchange), then the
    ranks compare their range outcomes (a few integers each: gather(obj) ->
    list of every rank's obj, torch.distributed.all_gather_object by default).
    When a rank's range was inexact (first_inexact), that rank replays again
    from its sync_begin to the end of the file and every later rank drops its
    results, so the ranks' results, concatenated in rank order, are always
    gpk_replay_file's on the whole file. Returns (results, stats, info):
    info["first_packet"] is the global index of this rank's first packet,
    info["ranges"] every rank's range outputs, info["redo_rank"] the rank that
    replayed again (None when the split was exact), info["dropped"] whether
    this rank's results were dropped."""
    import os
    if gather is None:
        import torch.distributed as dist

        def gather(obj):
            if world == 1 and not dist.is_initialized():
                return [obj]
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out
    from . import _lib
    size = os.path.getsize(path)
    failed = None
    try:
        res, st = ctx.replay_file(parser, path, byte_range=file_range(size, rank, world), **kw)
        mine = dict(st["range"], packets=int(st["packets"]))
    except _lib.GpkError as e:
        # a range whose replay failed outright (for instance on a record longer
        # than the staging carry region) is inexact like one that did not end
        # cleanly: after a false start it is dropped, else (a redo, or a kept
        # last range) the failure is the whole file's and is raised below
        if not hasattr(e, "range"):
            raise
        failed = e
        res, st = None, dict(packets=0, error=str(e))
        mine = dict(e.range, clean=0, packets=0)
    ranges = gather(mine)
    f = first_inexact(ranges)
    dropped = False
    if failed is not None and (f is None or rank < f):  # kept as it is: the failure is the file's
        raise failed
    if f is not None and rank == f:
        res, st = ctx.replay_file(parser, path, byte_range=(ranges[f]["sync_begin"], 0), **kw)
        st["redo_first"] = dict(mine)
        mine = dict(st["range"], packets=int(st["packets"]))
    elif f is not None and rank > f:
        dropped = True
        res = None if res is None else {k: v[:0] for k, v in res.items()}
        st["packets"] = 0
        mine = dict(mine, packets=0)
    counts = gather(mine["packets"]) if f is not None else [r["packets"] for r in ranges]
    info = dict(first_packet=int(sum(counts[:rank])), ranges=ranges, redo_rank=f, dropped=dropped,
                packets_per_rank=[int(c) for c in counts])
    return res, st, info
