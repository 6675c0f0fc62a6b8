"""One capture file replayed by N callers (C5 at N GPUs):
gpk_replay_file_range gives each caller the pcapng blocks that start in its
synced byte range (include/gpk_capture.h). The callers' results, concatenated
in range order, must equal gpk_replay_file on the whole file bit for bit
(records, error arguments, flow hashes, capture info, capture lengths, the
reader's final error), either directly (every range but the last clean and
without a section / interface block) or after the documented redo of the first
inexact range (shard.first_inexact). The whole-file replay itself is pinned to
the reader and decode oracles by tests/test_replay_gpu.py; here it is checked
against them once more for the synthetic capture. Files: the C4 IMIX mix,
payloads holding fake EPB chains (the sync rule's false positives), both byte
orders, a new interface and blocks longer than a walk segment mid-file, a
second section, corrupted files, and more ranks than the file has blocks."""
import os

import numpy as np
import pytest

import pcapgen
from configs import CONFIGS, device_parser
from test_replay_gpu import block_starts, check, walk_capture

pytestmark = pytest.mark.gpu

KEYS = ("records", "err_args", "ci", "caplens")


def concat(parts):
    out = {k: np.concatenate([p[k] for p in parts]) for k in KEYS}
    out["flows"] = np.concatenate([p["flows"].reshape(3, -1) for p in parts], axis=1).reshape(-1)
    return out


def same(a, b):
    return all(np.array_equal(a[k], b[k]) for k in KEYS + ("flows",))


def split_replay(ctx, parser, path, world, **kw):
    """Every rank's range in this one process (the C logic the ranks run),
    with the redo of shard.replay_file_sharded; returns (concatenated results,
    the last contributing rank's stats, the per-rank range outputs, redo rank)."""
    from gopacket_amd import shard
    from gopacket_amd import _lib
    size = os.path.getsize(path)
    outs = []
    for r in range(world):
        try:
            outs.append(ctx.replay_file(parser, path, byte_range=shard.file_range(size, r, world), **kw))
        except _lib.GpkError as e:  # inexact, like an unclean end (shard.replay_file_sharded)
            assert r < world - 1 and hasattr(e, "range"), str(e)
            outs.append((None, dict(range=dict(e.range, clean=0))))
    ranges = [st["range"] for _, st in outs]
    for r in range(1, world):  # the cuts chain: a rank begins where the previous one had to end
        assert ranges[r]["sync_begin"] == ranges[r - 1]["sync_end"], ranges
    assert ranges[0]["sync_begin"] == 0 and ranges[-1]["sync_end"] == size
    f = shard.first_inexact(ranges)
    parts = [res for res, _ in outs]
    last = outs[-1][1]
    if f is not None:
        res, last = ctx.replay_file(parser, path, byte_range=(ranges[f]["sync_begin"], 0), **kw)
        parts = parts[:f] + [res]
    return concat(parts), last, ranges, f


def whole_and_split(ctx, path, worlds, cfg="statsassembly", expect_exact=True, **kw):
    parser = device_parser(CONFIGS[cfg])
    whole, st = ctx.replay_file(parser, path, **kw)
    seen = {}
    for world in worlds:
        got, last, ranges, f = split_replay(ctx, parser, path, world, **kw)
        assert same(got, whole), (world, f, ranges)
        assert last["error"] == st["error"] and last["reader_status"] == st["reader_status"], (world, last["error"])
        if expect_exact:
            assert f is None, (world, ranges)
        seen[world] = (f, ranges)
    return whole, st, seen


@pytest.fixture(scope="module")
def imix(tmp_path_factory):
    from gopacket_amd import _lib
    path = str(tmp_path_factory.mktemp("rng") / "imix.pcapng")
    assert _lib.synth_lib().gpk_synth_write_pcapng(path.encode(), 4, 31, 40000, 4) > 0
    return path


def test_range_imix(gpu_ctx, imix):
    """The C4 mix split 2, 3, 5 and 8 ways: exact without a redo, every range
    non-empty, and the whole replay equal to the oracles."""
    raw = open(imix, "rb").read()
    check(gpu_ctx, imix, raw, slot_bytes=1 << 20, slots=3, batch_pkts=5000)
    _, st, seen = whole_and_split(gpu_ctx, imix, (2, 3, 5, 8), slot_bytes=1 << 20, slots=3, batch_pkts=5000)
    assert st["error"] == "EOF" and st["packets"] == 40000
    for world, (_, ranges) in seen.items():
        assert all(g["sync_end"] > g["sync_begin"] for g in ranges), (world, ranges)
        assert all(g["clean"] for g in ranges), (world, ranges)


def test_range_default_opts_and_fields(gpu_ctx, imix):
    """Default slots and batches, and fields=True: the layer fields concatenate too."""
    parser = device_parser(CONFIGS["statsassembly"])
    whole, _ = gpu_ctx.replay_file(parser, imix, fields=True)
    from gopacket_amd import shard
    size = os.path.getsize(imix)
    parts = [gpu_ctx.replay_file(parser, imix, fields=True, byte_range=shard.file_range(size, r, 4))[0]
             for r in range(4)]
    assert same(concat(parts), whole)
    assert np.array_equal(np.concatenate([p["fields"] for p in parts]), whole["fields"])


def test_range_option_blocks_are_state(gpu_ctx, tmp_path):
    """An EPB with options and an interface statistics block change reader
    state a later block can read (NgReader reuses one option buffer: a
    zero-length option keeps the previous value, ngread.go:214-219), so the
    range holding either is not exact for the ranges after it; a name record
    changes nothing. Three files, one of each, split 2 ways with the block in
    the first half."""
    from gopacket_amd import synth
    parser = device_parser(CONFIGS["statsassembly"])
    for kind in ("options", "isb", "nrb"):
        raw = pcapgen.shb() + pcapgen.idb(1, 0)
        for i in range(4000):
            p = synth.packet(4, i)
            if i == 1000 and kind == "options":
                raw += pcapgen.epb(p, ts=i, options=pcapgen.opt(1, b"note") + pcapgen.end_opt())
            elif i == 1000 and kind == "isb":
                raw += pcapgen.isb(0, 5, options=pcapgen.opt(4, bytes(8)) + pcapgen.end_opt())
            elif i == 1000:
                raw += pcapgen.nrb([(1, b"\x0a\x00\x00\x01x\x00")])
            else:
                raw += pcapgen.epb(p, ts=i)
        path = tmp_path / ("%s.pcapng" % kind)
        path.write_bytes(raw)
        whole, _ = gpu_ctx.replay_file(parser, str(path))
        got, _, ranges, f = split_replay(gpu_ctx, parser, str(path), 2)
        assert same(got, whole), kind
        assert ranges[0]["clean"], kind
        assert ranges[0]["state_changed"] == (kind != "nrb") and f == (None if kind == "nrb" else 0), (kind, ranges)


@pytest.mark.parametrize("bo", ["<", ">"])
def test_range_fake_chains(gpu_ctx, tmp_path, bo):
    """Payloads with fake EPB chains, three interfaces, an EPB with options, a
    name record and a statistics block (walk_capture): cuts at many offsets,
    some landing inside the packets that hold the fake chains."""
    raw = walk_capture(bo)
    path = tmp_path / "walk.pcapng"
    path.write_bytes(raw)
    _, _, seen = whole_and_split(gpu_ctx, str(path), (2, 3, 7, 16), expect_exact=False, slot_bytes=1 << 18,
                                 slots=3, batch_pkts=3000)
    for world, (f, ranges) in seen.items():  # the file's three interfaces are its header: every cut finds a block
        assert all(g["sync_end"] > g["sync_begin"] for g in ranges), (world, ranges)
        # the EPB with options (packet 4000, ~1/3 in) and the statistics block (~3/4 in) are reader state
        assert f is not None and f < world - 1, (world, f)


def test_range_cut_inside_fake_chain(gpu_ctx, tmp_path):
    """A cut a few bytes before a fake EPB chain, 4-byte aligned inside a
    packet: the sync rule takes the fake chain, the range before it cannot end
    cleanly there (its reader meets the end inside the real block), and the
    redo from the first range's start makes the result exact."""
    from gopacket_amd import synth, shard
    rng = np.random.default_rng(9)
    fake = b"".join(pcapgen.epb(bytes(rng.integers(0, 256, 40, dtype=np.uint8))) for _ in range(5))
    raw = pcapgen.shb() + pcapgen.idb(1, 0)
    starts = []
    for i in range(3000):
        p = synth.packet(4, i)
        if i == 1500:
            p = p[:16] + fake + p[16:]  # data starts 28 bytes into the block: the chain at block + 44
        starts.append(len(raw))
        raw += pcapgen.epb(p, ts=i)
    path = tmp_path / "fake.pcapng"
    path.write_bytes(raw)
    p = starts[1500]
    parser = device_parser(CONFIGS["statsassembly"])
    whole, st = gpu_ctx.replay_file(parser, str(path))
    assert st["packets"] == 3000 and st["error"] == "EOF"
    cut = p + 28 + 8
    a, sa = gpu_ctx.replay_file(parser, str(path), byte_range=(0, cut))
    try:
        _, sb = gpu_ctx.replay_file(parser, str(path), byte_range=(cut, 0))
        rb = sb["range"]
    except Exception as e:  # the range that starts at the fake chain reads garbage: dropped anyway
        rb = e.range
    assert sa["range"]["sync_end"] == rb["sync_begin"] == p + 44  # the fake chain
    assert not sa["range"]["clean"]
    assert shard.first_inexact([sa["range"], rb]) == 0
    redo, _ = gpu_ctx.replay_file(parser, str(path), byte_range=(sa["range"]["sync_begin"], 0))
    assert same(redo, whole)


def test_range_new_interface_and_big_blocks(gpu_ctx, tmp_path):
    """A new interface block mid-file (the reader state changes: the rank that
    holds it is inexact for the ranks after it), blocks of 16-64 KiB and a name
    record (which changes no reader state)."""
    from gopacket_amd import synth
    rng = np.random.default_rng(11)
    raw = pcapgen.shb() + pcapgen.idb(1, 0)
    for i in range(20000):
        p = synth.packet(4, i)
        if i % 2500 == 17:
            p = p + bytes(rng.integers(0, 256, int(rng.integers(16, 64)) << 10, dtype=np.uint8))
        if i == 6000:
            raw += pcapgen.nrb([(1, b"\x0a\x00\x00\x01x\x00")])
        elif i == 15000:
            raw += pcapgen.idb(1, 0)
        else:
            raw += pcapgen.epb(p, iface=1 if i > 15000 and i % 2 else 0, ts=i)
    path = tmp_path / "iface.pcapng"
    path.write_bytes(raw)
    _, _, seen = whole_and_split(gpu_ctx, str(path), (2, 4, 6), expect_exact=False, slot_bytes=1 << 20, slots=3,
                                 batch_pkts=4096)
    idb_at = raw.index(pcapgen.idb(1, 0), 100)  # the second interface block
    for world, (f, ranges) in seen.items():
        holder = [k for k, g in enumerate(ranges) if g["sync_begin"] <= idb_at < g["sync_end"]]
        assert holder and ranges[holder[0]]["state_changed"], (world, ranges)
        assert f == (holder[0] if holder[0] < world - 1 else None), (world, f, holder)


def test_range_two_sections_and_tiny_file(gpu_ctx, tmp_path):
    """SPB/PB/EPB, statistics, name records and a second section in the other
    byte order, 40 packets split up to 16 ways (most ranges empty)."""
    import pktutil
    g = pktutil.golden()
    pk = [bytes.fromhex(v["hex"]) for k, v in sorted(g.items()) if "hex" in v][:40]
    raw = pcapgen.shb() + pcapgen.idb(1, 0) + b"".join(pcapgen.epb(p, ts=i) for i, p in enumerate(pk[:10]))
    raw += pcapgen.nrb([(1, b"\x0a\x00\x00\x01x\x00")]) + b"".join(pcapgen.spb(p) for p in pk[10:20])
    raw += pcapgen.isb(0, 5) + pcapgen.shb(">") + pcapgen.idb(1, 0, ">") + b"".join(
        pcapgen.pb(p, bo=">") for p in pk[20:])
    path = tmp_path / "mixed.pcapng"
    path.write_bytes(raw)
    whole_and_split(gpu_ctx, str(path), (2, 5, 16), expect_exact=False, slot_bytes=4096, slots=2, batch_pkts=3)


@pytest.mark.parametrize("seed", [0, 3, 6, 8, 10, 11])
def test_range_corrupt(gpu_ctx, tmp_path, seed):
    """The corrupted files of test_replay_gpu.test_replay_device_walk_corrupt
    (the same seeds and flips: block types, lengths, interface ids, capture
    lengths, trailers, packet bytes; seeds >= 8 big-endian): the reader's
    desync or error lands in some range; the concatenation, after the redo, is
    still the whole replay, including its final error."""
    bo = ">" if seed >= 8 else "<"
    raw = bytearray(walk_capture(bo))
    blocks = block_starts(bytes(raw), bo)[4:]
    rng = np.random.default_rng(1000 + seed)
    for _ in range(int(rng.integers(1, 5))):
        p, L = blocks[int(rng.integers(0, len(blocks)))]
        field = int(rng.integers(0, 7))
        lo = 0 if bo == "<" else 3
        pos = [p + lo, p + 4 + lo, p + 8 + lo, p + 20 + lo, p + 24 + lo, p + L - 4 + lo,
               p + 28 + int(rng.integers(0, max(1, L - 32)))][field]
        raw[pos] ^= int(rng.integers(1, 256)) if field != 1 else int(rng.integers(1, 256)) & 0xFC | 4
    path = tmp_path / "corrupt.pcapng"
    path.write_bytes(bytes(raw))
    whole_and_split(gpu_ctx, str(path), (2, 3, 8), expect_exact=False)


def test_range_unsupported(gpu_ctx, tmp_path, imix):
    """Classic pcap and gzip files are replayed whole only."""
    import gzip
    from gopacket_amd import _lib, synth
    parser = device_parser(CONFIGS["statsassembly"])
    q = tmp_path / "x.pcap"
    q.write_bytes(pcapgen.pcap_file([synth.packet(4, i) for i in range(100)]))
    z = tmp_path / "x.pcapng.gz"
    z.write_bytes(gzip.compress(open(imix, "rb").read()[:100000]))
    for p in (q, z):
        with pytest.raises(_lib.GpkError, match="uncompressed pcapng"):
            gpu_ctx.replay_file(parser, str(p), byte_range=(0, 1000))


def _sharded_rank(rank, world, port, paths, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from gopacket_amd import engine, shard
    ctx = engine.Context(0)
    parser = device_parser(CONFIGS["statsassembly"])
    out = []
    for path in paths:
        res, st, info = shard.replay_file_sharded(ctx, parser, path, rank, world)
        out.append((res, st.get("error"), info))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_two_ranks_gloo(gpu_ctx, tmp_path, imix):
    """shard.replay_file_sharded in two processes (gloo, both on the one GPU):
    each rank replays its range and the ranks exchange only their range
    outcomes; the two ranks' results in rank order equal the whole replay, on
    the IMIX capture (an exact split) and on a corrupted capture and one with a
    new interface mid-file (where a redo may be needed)."""
    import socket
    import torch.multiprocessing as mp
    from test_shard_dist_gpu import _free_port
    raw = bytearray(walk_capture("<"))
    blocks = block_starts(bytes(raw))[4:]
    p, L = blocks[len(blocks) // 3]
    raw[p + 4] ^= 0x40  # a block length: the reader desynchronises a third of the way in
    bad = tmp_path / "bad.pcapng"
    bad.write_bytes(bytes(raw))
    from gopacket_amd import synth
    iface = pcapgen.shb() + pcapgen.idb(1, 0) + b"".join(
        pcapgen.epb(synth.packet(4, i), ts=i) if i != 2000 else pcapgen.idb(1, 0) for i in range(8000))
    ifp = tmp_path / "iface.pcapng"
    ifp.write_bytes(iface)
    paths = [imix, str(bad), str(ifp)]
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sharded_rank, args=(r, world, port, paths, q)) for r in range(world)]
    for pr in ps:
        pr.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for pr in ps:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    parser = device_parser(CONFIGS["statsassembly"])
    for k, path in enumerate(paths):
        whole, st = gpu_ctx.replay_file(parser, path)
        parts = [got[r][k][0] for r in range(world) if got[r][k][0] is not None]
        assert same(concat(parts), whole), (path, [got[r][k][2] for r in range(world)])
        infos = [got[r][k][2] for r in range(world)]
        assert infos[1]["first_packet"] == infos[0]["packets_per_rank"][0]
        last = max(r for r in range(world) if not infos[r]["dropped"])
        assert got[last][k][1] == st["error"], (path, got[last][k][1], st["error"])
        if k == 0:
            assert infos[0]["redo_rank"] is None
        if k == 2:  # the new interface is in rank 0's half: rank 0 redoes to the end, rank 1 is dropped
            assert infos[0]["redo_rank"] == 0 and infos[1]["dropped"]
