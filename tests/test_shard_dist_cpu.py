"""The N>1 path on CPU: world_size-2 and -4 gloo ranks, byte-balanced shards of one
IMIX batch, per-rank decode (oracle as the CPU stand-in for the device),
results gathered and compared with a single-rank decode; max-over-ranks timing."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from gopacket_amd import shard

DEC = ["ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP", "PAYLOAD"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gopacket_amd import synth
    from oracle import oracle as O
    d, o, c = synth.host_batch(synth.C4_IMIX, 0, 6000)
    cuts = shard.byte_balanced_bounds(c, world)
    lo, hi = cuts[rank], cuts[rank + 1]
    sub_o = o[lo:hi] - (o[lo] if hi > lo else 0)
    sub_d = d[int(o[lo]):int(o[hi - 1] + c[hi - 1]) + 16]
    r = O.OracleParser(17, DEC).decode(sub_d, sub_o, c[lo:hi], layouts=False)
    recs = [None] * world
    dist.all_gather_object(recs, (lo, hi, r["records"].tobytes()))
    t = shard.max_over_ranks(1.0 + rank, world)
    if rank == 0:
        q.put((recs, t, [int(c[cuts[k]:cuts[k + 1]].sum()) for k in range(world)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_rank_shards_concatenate_to_single_rank_result(world):
    from gopacket_amd import synth
    from oracle import oracle as O
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    recs, t, bytes_per_rank = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    d, o, c = synth.host_batch(synth.C4_IMIX, 0, 6000)
    whole = O.OracleParser(17, DEC).decode(d, o, c, layouts=False)["records"].tobytes()
    assert b"".join(x[2] for x in sorted(recs)) == whole
    assert t == float(world)  # slowest rank
    assert max(bytes_per_rank) - min(bytes_per_rank) <= 1518
