"""The N>1 path through libgpk on the GPU: world-2 gloo ranks (both on
cuda:0, the box has one GPU) each generate and decode their byte-balanced
shard of one IMIX batch through the C ABI; the gathered results must equal a
single-rank decode of the whole batch bit for bit (and the oracle on a
sample). Then bench.py itself under torchrun with 2 ranks: the multi-rank
bench path (barriers, max over ranks, strong-scaling shards)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEC = ("Ethernet", "Dot1Q", "IPv4", "IPv6", "IPv6ExtensionSkipper", "TCP", "UDP", "Payload")
N = 300000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _caplens(n):
    from gopacket_amd import _lib
    caps = np.zeros(n, np.uint32)
    _lib.synth_lib().gpk_synth_batch_host(4, 0, n, None, None, caps.ctypes.data)
    return caps


def _decode(first, n):
    import torch
    from gopacket_amd import engine, synth
    ctx = engine.Context(0)
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in DEC])
    d, o, c = synth.device_batch(4, first, n)
    rec = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
    fl = torch.zeros(3 * n, dtype=torch.int64, device="cuda")
    ctx.decode_device(parser, d, o, c, rec, err, fl)
    torch.cuda.synchronize()
    return rec.cpu().numpy().tobytes(), fl.cpu().numpy().reshape(3, n), err.cpu().numpy()


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from gopacket_amd import shard
    cuts = shard.byte_balanced_bounds(_caplens(N), world)
    lo, hi = cuts[rank], cuts[rank + 1]
    rec, fl, err = _decode(lo, hi - lo)
    t = shard.max_over_ranks(1.0 + rank, world, device="cuda")
    parts = [None] * world
    dist.all_gather_object(parts, (lo, hi, rec, fl, err))
    if rank == 0:
        q.put((parts, t))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_device_shards_concatenate_to_single_rank_result():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    parts, t = q.get(timeout=240)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert t == 2.0
    parts.sort(key=lambda x: x[0])
    assert parts[0][0] == 0 and parts[-1][1] == N and parts[0][1] == parts[1][0]
    rec, fl, err = _decode(0, N)
    assert b"".join(x[2] for x in parts) == rec
    assert np.array_equal(np.concatenate([x[3] for x in parts], axis=1), fl)
    assert np.array_equal(np.concatenate([x[4] for x in parts]), err)
    # and a sample against the oracle
    from gopacket_amd import _lib, synth
    from oracle import oracle as O
    idx = np.unique(np.random.default_rng(3).integers(0, N, 3000))
    pk = [synth.packet(4, int(i)) for i in idx]
    cap = np.array([len(x) for x in pk], np.uint32)
    off = np.concatenate([[0], np.cumsum(cap[:-1], dtype=np.uint64)]).astype(np.uint64)
    ref = O.OracleParser(17, ["ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP", "PAYLOAD"]).decode(
        np.frombuffer(b"".join(pk) + bytes(16), np.uint8), off, cap, layouts=False)
    got = np.frombuffer(rec, np.uint8).reshape(N, 16)[idx].reshape(-1).view(_lib.RECORD_DTYPE)
    assert np.array_equal(got, ref["records"])


def test_bench_two_ranks_strong_and_weak():
    """bench.py's multi-rank branch as the driver invokes it: `python bench.py
    --gpus 2 ...` with no launcher (bench.py starts torch.distributed.run as
    a child, 2 ranks, gloo, both on the box's one GPU)."""
    env = dict(os.environ, OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo",
           "--same-device", "--configs", "c3,c4s", "--packets", str(1 << 20), "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--c5", "0.03", "--no-probe"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["steps"] == 2 and r["scaling"] == "weak"
    assert r["dist_backend"] == "gloo"
    assert r["parity"].startswith("bit-exact")
    ks = r["roofline"]["kernel_ms_ranks"]
    assert len(ks) == 2 and abs(r["roofline"]["kernel_ms"] - max(ks)) < 1e-3
    c = r["configs"]["c4s"]
    assert c["scaling"] == "strong" and c["total_packets"] == 1 << 20
    assert c["parity"].startswith("bit-exact") and 1.0 <= c["byte_balance"] < 1.001
    assert len(c["kernel_ms_ranks"]) == 2 and abs(c["kernel_ms"] - max(c["kernel_ms_ranks"])) < 1e-3
    assert r["roofline"]["kernel"].startswith("gpk::decode_kernel<true,false,true,false,")
    # the N>1 line is as strong as the N=1 line: every rank checks every packet of its
    # own shard against the oracle, runs the layer-fields row and its share of C5
    assert r["parity"].startswith("bit-exact on every rank")
    for row in (r["full_parity"], c["full_parity"]):
        assert row["result"].startswith("bit-exact on every rank (2 ranks"), row
        assert [x["rank"] for x in row["ranks"]] == [0, 1]
        assert all(x["result"].startswith("bit-exact (all %d packets" % x["packets"]) for x in row["ranks"]), row
        assert all("and the narrow form" in x["result"] for x in row["ranks"]), row
    assert r["narrow"]["kernel_ms"] > 0 and c["narrow"]["kernel_ms"] > 0
    assert sum(x["packets"] for x in c["full_parity"]["ranks"]) == 1 << 20
    assert [x["first_packet"] for x in r["full_parity"]["ranks"]] == [0, 1 << 20]
    f = r["fields"]
    assert len(f["ranks"]) == 2 and all(x["parity"].startswith("bit-exact") for x in f["ranks"]), f
    c5 = r["c5"]
    assert c5["parity"].startswith("bit-exact") and c5["packets"] == c5["file_packets"] > 0, c5
    assert [x["rank"] for x in c5["ranks"]] == [0, 1] and c5["ranks"][1]["first_packet"] == c5["ranks"][0]["packets"]
    assert c5["redo_rank"] is None and all(x["range"]["clean"] for x in c5["ranks"]), c5["ranks"]
    assert r["cpu_baseline"] is None and "N=1 only" in r["cpu_baseline_note"]

def test_bench_rccl_world_one():
    """bench.py's RCCL branch on a one-GPU box: torchrun with one rank and
    --force-dist, so init_process_group("nccl", device_id=...), the barriers
    and the max over ranks run through RCCL. Multi-GPU
    scaling itself stays unmeasured here (one GPU per box)."""
    env = dict(os.environ, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1", "--force-dist",
           "--configs", "c3,c2", "--packets", str(1 << 20), "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--c5", "0", "--no-full-parity"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    line = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
    r = json.loads(line)
    assert r["dist_backend"] == "nccl"
    assert r["n_gpus"] == 1 and r["steps"] == 3 and r["scaling"] == "weak" and r["value"] > 0
    assert r["parity"].startswith("bit-exact") and r["configs"]["c2"]["parity"].startswith("bit-exact")
    # the probes ran: the streaming read and each config's memory skeleton beside its kernel
    for row in (r["roofline"], r["configs"]["c2"]):
        assert row["probe_read_GBps"] > 0 and row["skeleton_ms"] > 0 and 0.2 < row["of_skeleton"] < 5
