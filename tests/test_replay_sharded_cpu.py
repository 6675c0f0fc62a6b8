"""shard.replay_file_sharded's protocol on CPU (gloo, world size 2): each rank
replays its byte range, the ranks swap their range outcomes, and an inexact
split (a range that did not end cleanly, changed the reader state, or failed)
is redone by the first inexact rank from its sync_begin to the end of the file
while the later ranks drop theirs. A fake context stands in for the library:
the file is a list of blocks, and a range replay returns the blocks that start
in it (gpk_replay_file_range's contract, include/gpk_capture.h)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from gopacket_amd import shard


class FakeCtx:
    """A 'file' of blocks at the given starts; sync(X) = first block start >= X
    that is not in `fake` (and the fake positions, which are inside blocks,
    when X falls right before one). A range's reader is clean when its end is
    a real block start; state changes at blocks listed in `idb`; `raise_at`
    makes a range that starts there fail outright."""

    def __init__(self, starts, size, fake=(), idb=(), raise_at=()):
        self.starts, self.size, self.fake, self.idb, self.raise_at = list(starts), size, set(fake), set(idb), set(raise_at)
        self.calls = []

    def sync(self, x):
        cands = sorted(set(self.starts) | self.fake)
        for p in cands:
            if p >= x:
                return p
        return self.size

    def replay_file(self, parser, path, byte_range=None, **kw):
        from gopacket_amd import _lib
        b0, e0 = byte_range
        b = 0 if b0 == 0 else self.sync(b0)
        e = self.size if e0 == 0 else max(b, self.sync(e0))
        self.calls.append((b0, e0))
        rng = dict(begin=b0, end=e0, header_end=0, sync_begin=b, sync_end=e,
                   clean=int(e == self.size or e in self.starts), state_changed=0)
        if b in self.raise_at:
            err = _lib.GpkError("gpk_replay_file: -5 capture record larger than the staging carry region")
            err.range = dict(rng, clean=0)
            raise err
        pk = [s for s in self.starts if b <= s < e] if b in self.starts or b == 0 else [b + 1, b + 2]
        rng["state_changed"] = int(any(s in self.idb for s in pk))
        res = dict(records=np.array(pk, np.int64))
        return res, dict(packets=len(pk), error="EOF", range=rng)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, scenarios, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    for sc in scenarios:
        ctx = FakeCtx(**sc)
        path = os.devnull
        size = sc["size"]
        orig = os.path.getsize
        os.path.getsize = lambda p, size=size: size  # the fake file's size
        try:
            res, st, info = shard.replay_file_sharded(ctx, None, path, rank, world)
        finally:
            os.path.getsize = orig
        out.append((res["records"].tolist() if res else [], info, ctx.calls))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


STARTS = list(range(0, 1000, 40))  # blocks every 40 bytes
SCENARIOS = [
    dict(starts=STARTS, size=1000),                              # exact
    dict(starts=STARTS, size=1000, fake=[504]),                  # rank 0 ends inside a block: redo
    dict(starts=STARTS, size=1000, idb=[120]),                   # a new interface in rank 0's range: redo
    dict(starts=STARTS, size=1000, idb=[720]),                   # ... in the last rank's range: exact
    dict(starts=STARTS, size=1000, fake=[504], raise_at=[504]),  # rank 1's range fails outright
]


def test_replay_file_sharded_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, SCENARIOS, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = STARTS
    for k, sc in enumerate(SCENARIOS):
        recs = got[0][k][0] + got[1][k][0]
        assert recs == whole, (k, recs)
        i0, i1 = got[0][k][1], got[1][k][1]
        assert i1["first_packet"] == len(got[0][k][0])
        redo = None if k in (0, 3) else 0
        assert i0["redo_rank"] == i1["redo_rank"] == redo, (k, i0, i1)
        assert i1["dropped"] == (redo == 0)
        if redo == 0:  # rank 0 replayed again from its start to the end of the file
            assert got[0][k][2][-1] == (0, 0)


def test_file_range_and_first_inexact():
    assert [shard.file_range(1000, r, 3) for r in range(3)] == [(0, 333), (333, 666), (666, 0)]
    ok = dict(clean=1, state_changed=0)
    assert shard.first_inexact([ok, ok, dict(clean=0, state_changed=1)]) is None  # the last rank's end is the file's
    assert shard.first_inexact([ok, dict(clean=0, state_changed=0), ok]) == 1
    assert shard.first_inexact([dict(clean=1, state_changed=1), ok]) == 0
