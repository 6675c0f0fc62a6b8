#!/usr/bin/env python3
"""Benchmark: device-resident Eth/IPv4/TCP decode + checksum + flow hash.

A step = one gpk_decode_batch over one per-GPU batch already resident in HBM
(BASELINE.json configs[2], "C3": 64 M synthetic 1500 B Eth/IPv4/TCP packets,
full TCP/IP checksum + flow hash). Secondary configs C2 (64 B UDP, IPv4
checksum) and C4 (IMIX + VLAN + IPv6, all checksums and hashes) are measured
in the same run and reported under "configs".

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Multi-GPU: every rank generates and decodes its own shard (packets
[rank*n, (rank+1)*n)); no collective on the data path ("scaling": "weak").
Timing: barrier + synchronize on both sides of exactly K steps, max over ranks.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
INDEX_BYTES = 12       # u64 offset + u32 caplen per packet

CONFIGS = {
    # BASELINE configs[0]: the reference's CPU-runnable case, pcap/test_ethernet.pcap's 10
    # packets replayed 10^6 times (benchmark.go -repeat), as decode_test.go:192's parser
    "c1": dict(pcap="tests/golden/test_ethernet.pcap", packets=10_000_000,
               decoders=("Ethernet", "IPv4", "TCP", "Payload"), outputs=3,
               workload="C1: test_ethernet.pcap (10 packets) replayed 1e6 times, Eth/IPv4/TCP decode + IPv4/TCP checksums"),
    "c3": dict(synth=3, decoders=("Ethernet", "IPv4", "TCP", "Payload"), outputs=7,
               workload="C3: 64M x 1500B Eth/IPv4/TCP, IPv4+TCP checksum, link/net/transport FastHash"),
    "c2": dict(synth=2, decoders=("Ethernet", "IPv4", "UDP", "Payload"), outputs=1,
               workload="C2: 64M x 64B Eth/IPv4/UDP, header decode + IPv4 checksum"),
    # diagnostics (not bench lines): C3 bytes with the L4 checksum and flows off
    "c3h": dict(synth=3, decoders=("Ethernet", "IPv4", "TCP", "Payload"), outputs=1,
                workload="C3 packets, headers + IPv4 checksum only (diagnostic)"),
    "c4": dict(synth=4, decoders=("Ethernet", "Dot1Q", "IPv4", "IPv6", "IPv6ExtensionSkipper", "TCP", "UDP",
                                  "Payload"), outputs=7,
               workload="C4: 64M IMIX 64/594/1518 7:4:1, 40% Dot1Q/QinQ, 20% IPv6, all checksums + hashes"),
}
# diagnostics (not bench lines): C4 / C1 with subsets of the outputs (1 IPv4 checksum, 2 L4
# checksum, 4 flow hashes), to split the kernel time between the parse and each output
for _o in (1, 3, 5):
    CONFIGS["c4x%d" % _o] = dict(CONFIGS["c4"], outputs=_o, workload="C4 packets, outputs %d (diagnostic)" % _o)
CONFIGS["c1x1"] = dict(CONFIGS["c1"], outputs=1, workload="C1 packets, IPv4 checksum only (diagnostic)")
CONFIGS["c4x0"] = dict(CONFIGS["c4"], outputs=0, workload="C4 packets, decode only (diagnostic)")
CONFIGS["c2x0"] = dict(CONFIGS["c2"], outputs=0, workload="C2 packets, decode only (diagnostic)")
# C4's IMIX packets through a parser with no IPv6 decoder: the dword-window kernel (decode_kernel<..., 4>)
# on waves of mixed sizes (diagnostic)
CONFIGS["c4m"] = dict(CONFIGS["c4"], decoders=("Ethernet", "Dot1Q", "IPv4", "TCP", "UDP", "Payload"),
                      workload="C4 packets, parser without IPv6 (diagnostic: dword-window kernel)")
# BASELINE configs[3] as written: ONE 64M IMIX batch split across the ranks at byte-balanced
# cuts (shard.byte_balanced_bounds; strong scaling, run by default when world > 1)
CONFIGS["c4s"] = dict(CONFIGS["c4"], strong=True,
                      workload="C4 strong: one 64M IMIX batch sharded over the ranks (byte-balanced cuts)")


# engine decoder names -> oracle decoder names
ORACLE_DEC = {"Ethernet": "ETHERNET", "Dot1Q": "DOT1Q", "IPv4": "IPV4", "IPv6": "IPV6",
              "IPv6ExtensionSkipper": "IPV6_EXT", "TCP": "TCP", "UDP": "UDP", "Payload": "PAYLOAD"}


def dist_init(backend="nccl", same_device=False, force=False):
    """One process per GPU (torchrun env). backend "nccl" is RCCL on ROCm;
    "gloo" + same_device=True rehearses N ranks on one GPU (tests only).
    force=True initialises the process group at world size 1 too, so the
    barrier and the max-over-ranks run through the backend (tests only)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1 or force:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_plan(gpus, environ, argv, port=None):
    """How `bench.py --gpus N` runs (one process per GPU, the contract's
    launch). Decided before anything touches the GPU:
    - a launcher set WORLD_SIZE: this process is one rank; WORLD_SIZE must
      equal N (a mismatch is an error, not a silent world-size-1 run);
    - no launcher and N == 1: run here;
    - no launcher and N > 1: start `python -m torch.distributed.run
      --nproc-per-node N bench.py <same args>` as a CHILD process (never an
      exec) and relay its output.
    Returns ("inproc", None) or ("spawn", argv of the child)."""
    world = environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%s (launch one rank per GPU)" % (gpus, world))
        return "inproc", None
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if gpus == 1:
        return "inproc", None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port or free_port()),
           os.path.join(ROOT, "bench.py")] + list(argv)
    return "spawn", cmd


def spawn_ranks(cmd):
    """Run the torchrun child, pass its stdout through line by line (rank 0
    prints the one JSON line) and return its exit status; a run that ends
    without a JSON line is a failure."""
    import signal
    import subprocess
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "16")  # (torchrun would set 1 and warn; the ranks' host work is the parity check)
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)

    def on_term(signum, frame):  # a driver's timeout: end the ranks too, not just this parent
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, on_term)
    lines = 0
    try:
        for line in p.stdout:
            if line.startswith("{"):
                lines += 1
            sys.stdout.write(line)
            sys.stdout.flush()
        rc = p.wait()
    except BaseException:
        p.terminate()
        p.wait(timeout=30)
        raise
    if rc == 0 and lines != 1:
        sys.stderr.write("bench.py: the multi-rank run printed %d JSON lines, not 1\n" % lines)
        return 1
    return rc


def gather_ranks(x, world):
    """Every rank's value of x, in rank order (None at world size 1 without a
    process group)."""
    import torch.distributed as dist
    if world == 1 and not dist.is_initialized():
        return None
    out = [None] * world
    dist.all_gather_object(out, round(float(x), 4))
    return out


def gather_obj(x, world):
    """Every rank's x (any picklable object), in rank order; [x] at world size
    1 without a process group."""
    import torch.distributed as dist
    if world == 1 and not dist.is_initialized():
        return [x]
    out = [None] * world
    dist.all_gather_object(out, x)
    return out


def rank_threads():
    """Host threads one rank may use for its parity checks: the job's CPU
    share divided among the ranks on this node (torchrun's LOCAL_WORLD_SIZE),
    at most OMP_NUM_THREADS (a per-process setting)."""
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    per = max(2, host_cores()[2] // local)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return min(per, int(omp)) if omp.isdigit() and int(omp) > 0 else per


def barrier(world):
    import torch
    import torch.distributed as dist
    if world > 1 or dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()


def probe_read(data, nbytes, steps, stream):
    """Achievable streaming-read rate over the same buffer (GB/s): a kernel
    that only loads the bytes (gpk_probe_read), timed like the decode."""
    import torch
    from gopacket_amd import _lib
    S = _lib.synth_lib()
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    blocks = 256 * 8

    def go():
        rc = S.gpk_probe_read(data.data_ptr(), nbytes, sink.data_ptr(), blocks, stream.cuda_stream)
        assert rc == 0

    go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        go()
    e1.record(stream)
    torch.cuda.synchronize()
    return (nbytes & ~15) / (e0.elapsed_time(e1) / steps * 1e-3) / 1e9


def run_config(name, n, steps, warmup, rank, world, ctx, check_sample=2048, probe=False, full_check=False,
               narrow=True):
    import torch
    from gopacket_amd import engine, shard, synth
    cfg = CONFIGS[name]
    kinds = [engine.DECODER_KINDS[d] for d in cfg["decoders"]]
    parser = engine.ParserConfig(17, kinds, outputs=cfg["outputs"])
    if "pcap" in cfg:
        n = cfg["packets"]
    strong = None
    if cfg.get("strong"):
        # every rank computes the same cuts from the batch's capture lengths
        # (deterministic per packet index) and generates only its own range
        caps = np.zeros(n, np.uint32)
        from gopacket_amd import _lib
        _lib.synth_lib().gpk_synth_batch_host(cfg["synth"], 0, n, None, None, caps.ctypes.data)
        cuts = shard.byte_balanced_bounds(caps, world)
        per = [int(caps[cuts[k]:cuts[k + 1]].sum(dtype=np.uint64)) for k in range(world)]
        strong = dict(total_packets=n, cuts=cuts, bytes_per_rank=per,
                      balance=round(max(per) / (sum(per) / world), 6))
        first, n = cuts[rank], cuts[rank + 1] - cuts[rank]
        del caps
    else:
        first, n = shard.weak_range(rank, n)
    stream = torch.cuda.current_stream()
    if "pcap" in cfg:
        data, off, cap = pcap_tiled(cfg["pcap"], n)
    else:
        data, off, cap = synth.device_batch(cfg["synth"], first, n, stream=stream)
    rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
    fl = torch.empty(3 * n, dtype=torch.int64, device="cuda") if cfg["outputs"] & 4 else None
    payload_bytes = int(cap.sum(dtype=torch.int64).item())
    kernel = ctx.kernel_name(parser, data, off, cap)
    blocks_per_cu = ctx.occupancy(parser, data, off, cap)
    torch.cuda.synchronize()

    def step():
        ctx.decode_device(parser, data, off, cap, rec, err, fl, stream=stream)

    for _ in range(warmup):
        step()
    # and at least ~50 ms of launches: a short kernel (C1: 0.3 ms) right after
    # its batch was generated runs ~20 % slower for its first ~10 ms of launches
    # (clock ramp), which 3 steps do not cover (tools/c1_diag.py)
    torch.cuda.synchronize()
    tw = time.perf_counter()
    while time.perf_counter() - tw < 0.05:
        for _ in range(4):
            step()
        torch.cuda.synchronize()
    barrier(world)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        step()
    e1.record(stream)
    barrier(world)
    wall = time.perf_counter() - t0
    kernel_ms_own = e0.elapsed_time(e1) / steps
    wall_max = shard.max_over_ranks(wall, world, device="cuda")
    # the slowest rank's kernel time (each rank's own, for the record)
    kernel_ms = shard.max_over_ranks(kernel_ms_own, world, device="cuda")
    kernel_ms_ranks = gather_ranks(kernel_ms_own, world)

    # the same decode with the 8-byte record (gpk_decode_batch_narrow, include/gpk.h gpk_record8), timed
    # the same way on its own outputs; the every-packet check below covers both forms
    nar = None
    if narrow:
        rec8 = torch.empty(n * 8, dtype=torch.uint8, device="cuda")
        wide = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
        err8 = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
        fl8 = torch.empty(3 * n, dtype=torch.int64, device="cuda") if fl is not None else None

        def nstep():
            ctx.decode_device_narrow(parser, data, off, cap, rec8, wide, err8, fl8, stream=stream)

        for _ in range(max(warmup, 2)):
            nstep()
        barrier(world)
        n0, n1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n0.record(stream)
        for _ in range(steps):
            nstep()
        n1.record(stream)
        barrier(world)
        nk = shard.max_over_ranks(n0.elapsed_time(n1) / steps, world, device="cuda")
        nar = dict(kernel_ms=nk, buffers=(rec8, wide, err8, fl8))

    probe_gbs = probe_read(data, payload_bytes, steps, stream) if probe else None
    skel_ms = skeleton_ms(cfg, data, off, cap, n, steps, stream) if probe and not strong else None
    parity = None
    if check_sample:
        parity = sample_parity(name, cfg, rec, fl, err, first, n, check_sample)
        if world > 1:
            every = gather_obj(parity, world)
            parity = ("bit-exact on every rank: " if all(p.startswith("bit-exact") for p in every)
                      else "MISMATCH on a rank: ") + "; ".join("rank %d %s" % (k, p) for k, p in enumerate(every))
    full = None
    if full_check:
        full, full_s = full_parity(name, cfg, data, off, cap, rec, fl, err, n, rank_threads(),
                                   narrow=nar["buffers"] if nar else None)
        full = dict(result=full, seconds=round(full_s, 2), threads=rank_threads())
        if world > 1:  # every rank checks its own shard; the line carries each rank's result
            full = dict(ranks=gather_obj(dict(full, rank=rank, first_packet=first, packets=n), world),
                        result=None, seconds=None)
            bad = [x for x in full["ranks"] if not x["result"].startswith("bit-exact")]
            full["result"] = ("bit-exact on every rank (%d ranks, %d packets)" % (world, sum(
                x["packets"] for x in full["ranks"]))) if not bad else "MISMATCH on rank(s) %s" % [x["rank"] for x in bad]
            full["seconds"] = max(x["seconds"] for x in full["ranks"])
    if nar:
        nar.pop("buffers")
    res = dict(full_parity=full, n=n, payload_bytes=payload_bytes, wall_s=wall_max, kernel_ms=kernel_ms, narrow=nar,
               kernel_ms_ranks=kernel_ms_ranks,
               algo_bytes=payload_bytes + INDEX_BYTES * n, parity=parity, probe_gbs=probe_gbs, skeleton_ms=skel_ms,
               strong=strong,
               kernel=kernel, blocks_per_cu=blocks_per_cu)
    del data, off, cap, rec, err, fl
    if narrow:
        del rec8, wide, err8, fl8
    torch.cuda.empty_cache()
    return res


# Bytes a decode writes per packet, and whether it streams the packet bytes
# (an L4 checksum), for its memory skeleton (tools/skeleton_all.py)
def skeleton_shape(cfg):
    return (16 + (24 if cfg["outputs"] & 4 else 0)), bool(cfg["outputs"] & 2)


def skeleton_ms(cfg, data, off, cap, n, steps, stream, wbytes=None):
    """The decode's memory skeleton on the same batch (gpk_probe_skeleton_idx:
    index, header windows, the wave's stream, the bytes the decode writes;
    none of its work), timed like the decode."""
    import torch
    from gopacket_amd import _lib
    S = _lib.synth_lib()
    w, streamed = skeleton_shape(cfg)
    wbytes = w if wbytes is None else wbytes
    wbuf = torch.empty(wbytes * n, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")

    def go():
        assert S.gpk_probe_skeleton_idx(data.data_ptr(), off.data_ptr(), cap.data_ptr(), n, wbuf.data_ptr(),
                                        wbuf.numel(), wbytes, 2 | (0 if streamed else 64), sink.data_ptr(),
                                        stream.cuda_stream) == 0

    go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        go()
    e1.record(stream)
    torch.cuda.synchronize()
    del wbuf
    return e0.elapsed_time(e1) / steps


def pcap_packets(path):
    """The packets of a classic little-endian pcap file (bench input, not the reader under test)."""
    import struct
    raw = open(os.path.join(ROOT, path), "rb").read()
    pos, out = 24, []
    while pos + 16 <= len(raw):
        caplen = struct.unpack_from("<I", raw, pos + 8)[0]
        out.append(raw[pos + 16:pos + 16 + caplen])
        pos += 16 + caplen
    return out


def pcap_tiled(path, n):
    """Device batch of n packets: the file's packets repeated in order."""
    import torch
    pk = pcap_packets(path)
    one = np.frombuffer(b"".join(pk), np.uint8)
    caps = np.array([len(p) for p in pk], np.int64)
    reps = (n + len(pk) - 1) // len(pk)
    cap = np.tile(caps, reps)[:n]
    off = np.concatenate([[0], np.cumsum(cap[:-1])])
    data = np.zeros(int(cap.sum()) + 256, np.uint8)
    data[:len(one) * (n // len(pk))] = np.tile(one, n // len(pk))
    rest = n % len(pk)
    if rest:
        tail = np.frombuffer(b"".join(pk[:rest]), np.uint8)
        data[len(one) * (n // len(pk)):len(one) * (n // len(pk)) + len(tail)] = tail
    return (torch.from_numpy(data).cuda(), torch.from_numpy(off).cuda(),
            torch.from_numpy(cap.astype(np.int32)).cuda())


def sample_parity(name, cfg, rec, fl, err, first, n, k):
    """Check k sampled packets of the device result against the CPU oracle."""
    from gopacket_amd import _lib, synth
    from oracle import oracle as O
    rng = np.random.default_rng(first + 17)
    idx = np.unique(np.concatenate([rng.integers(0, n, k), [0, n - 1]]))
    if "pcap" in cfg:
        src = pcap_packets(cfg["pcap"])
        pk = [src[int(i) % len(src)] for i in idx]
    else:
        pk = [synth.packet(cfg["synth"], first + int(i)) for i in idx]
    cap = np.array([len(x) for x in pk], np.uint32)
    off = np.concatenate([[0], np.cumsum(cap[:-1], dtype=np.uint64)]).astype(np.uint64)
    data = np.frombuffer(b"".join(pk) + bytes(16), np.uint8)
    dec = [{"Ethernet": "ETHERNET", "Dot1Q": "DOT1Q", "IPv4": "IPV4", "IPv6": "IPV6",
            "IPv6ExtensionSkipper": "IPV6_EXT", "TCP": "TCP", "UDP": "UDP", "Payload": "PAYLOAD"}[d]
           for d in cfg["decoders"]]
    ref = O.OracleParser(17, dec, outputs=cfg["outputs"]).decode(data, off, cap, layouts=False)
    import torch
    ti = torch.from_numpy(idx.astype(np.int64)).cuda()
    got = rec.view(n, 16)[ti].cpu().numpy().reshape(-1).view(_lib.RECORD_DTYPE)
    ok = bool(np.array_equal(got, ref["records"]))
    if fl is not None:
        gf = torch.stack([fl[ti], fl[n + ti], fl[2 * n + ti]]).cpu().numpy().view(np.uint64).reshape(-1)
        ok = ok and bool(np.array_equal(gf, ref["flows"]))
    return "%s (%d sampled packets vs oracle)" % ("bit-exact" if ok else "MISMATCH", len(idx))


def full_parity(name, cfg, data, off, cap, rec, fl, err, n, threads, chunk=1 << 20, narrow=None):
    """Every packet of the device batch against the CPU oracle (SURVEY.md §8c
    at full size): chunks of the batch's own bytes and index are copied back,
    decoded by oracle/gpk_oracle.c on `threads` host threads, and the records,
    error arguments and flows compared bit for bit with the device outputs.
    narrow=(records8, wide, err_args, flows) of gpk_decode_batch_narrow on the
    same batch: checked in the same pass against the oracle's narrow form
    (every record8 and the whole side array, zero where no record widened).
    Returns (summary string, seconds)."""
    from gopacket_amd import _lib
    from oracle import oracle as O
    dec = [{"Ethernet": "ETHERNET", "Dot1Q": "DOT1Q", "IPv4": "IPV4", "IPv6": "IPV6",
            "IPv6ExtensionSkipper": "IPV6_EXT", "TCP": "TCP", "UDP": "UDP", "Payload": "PAYLOAD"}[d]
           for d in cfg["decoders"]]
    p = O.OracleParser(17, dec, outputs=cfg["outputs"])
    t0 = time.perf_counter()
    bad, first_bad = 0, None
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        o = off[a:b].cpu().numpy().astype(np.uint64)
        c = cap[a:b].cpu().numpy().astype(np.uint32)
        lo, hi = int(o.min()), int((o + c).max())
        host = np.empty(hi - lo + 16, np.uint8)
        host[:hi - lo] = data[lo:hi].cpu().numpy()
        host[hi - lo:] = 0
        ref = p.decode(host, o - np.uint64(lo), c, nthreads=threads, layouts=False)
        got = rec[a * 16:b * 16].cpu().numpy().view(_lib.RECORD_DTYPE)
        ok = got == ref["records"]
        ge = err[2 * a:2 * b].cpu().numpy().view(np.uint32).reshape(-1, 2)
        ok &= (ge == ref["err_args"].reshape(-1, 2)).all(axis=1)
        if fl is not None:
            rf = ref["flows"].reshape(3, -1)
            for k in range(3):
                ok &= fl[k * n + a:k * n + b].cpu().numpy().view(np.uint64) == rf[k]
        if narrow is not None:
            r8, w8, e8, f8 = narrow
            rn = p.decode_narrow(host, o - np.uint64(lo), c, nthreads=threads)
            g8 = r8[a * 8:b * 8].cpu().numpy().view(np.uint64)
            ok &= g8 == rn["records8"].view(np.uint64)
            gw = w8[a * 16:b * 16].cpu().numpy().view(np.uint64).reshape(-1, 2)
            ok &= (gw == rn["wide"].view(np.uint64).reshape(-1, 2)).all(axis=1)
            ok &= (e8[2 * a:2 * b].cpu().numpy().view(np.uint32).reshape(-1, 2) ==
                   rn["err_args"].reshape(-1, 2)).all(axis=1)
            if f8 is not None:
                rf = rn["flows"].reshape(3, -1)
                for k in range(3):
                    ok &= f8[k * n + a:k * n + b].cpu().numpy().view(np.uint64) == rf[k]
        nb = int((~ok).sum())
        if nb and first_bad is None:
            first_bad = a + int(np.argmin(ok))
        bad += nb
    secs = time.perf_counter() - t0
    if bad:
        return "MISMATCH (%d of %d packets differ from the oracle, first at %d)" % (bad, n, first_bad), secs
    return "bit-exact (all %d packets vs oracle: records, error arguments%s%s)" % (
        n, ", flows" if fl is not None else "",
        "; and the narrow form: records8, side array, error arguments%s" % (", flows" if fl is not None else "")
        if narrow is not None else ""), secs


def host_cores():
    """(threads used, nproc, CPU share, CPU model). The GPU box gives a
    process a share of the host (a cgroup CPU quota, cpu.max, and
    OMP_NUM_THREADS: 16 cores per GPU on the driver's boxes, with every CPU of
    the machine in the affinity mask) while nproc counts the whole machine; the
    parallel CPU baseline runs one thread per core of the share."""
    share = len(os.sched_getaffinity(0))
    try:  # a cgroup v2 CPU quota ("quota period"): the box's share of a larger machine
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max" and int(p) > 0:
            share = min(share, -(-int(q) // int(p)))
    except (OSError, ValueError):
        pass
    nproc = os.cpu_count() or share
    omp = os.environ.get("OMP_NUM_THREADS", "")
    threads = min(share, int(omp)) if omp.isdigit() and int(omp) > 0 else share
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return threads, nproc, share, model


def host_sample(name, batch):
    """A packed host batch of the config's first `batch` packets (synthetic
    generator, or the pcap's packets tiled), as the CPU baseline's input."""
    from gopacket_amd import synth
    cfg = CONFIGS[name]
    if "synth" in cfg:
        return synth.host_batch(cfg["synth"], 0, batch)
    pk = pcap_packets(cfg["pcap"])
    one = b"".join(pk)
    reps = batch // len(pk)
    cap = np.tile(np.array([len(p) for p in pk], np.uint32), reps)
    off = np.concatenate([[0], np.cumsum(cap[:-1], dtype=np.uint64)]).astype(np.uint64)
    return np.frombuffer(one * reps + bytes(16), np.uint8), off, cap


def oracle_rate(name, data, off, cap, threads, secs):
    """The oracle (CPU restatement, oracle/) over a host batch, replayed until
    `secs` elapse: (Mpkts/s, replays, seconds)."""
    from oracle import oracle as O
    cfg = CONFIGS[name]
    dec = [{"Ethernet": "ETHERNET", "Dot1Q": "DOT1Q", "IPv4": "IPV4", "IPv6": "IPV6",
            "IPv6ExtensionSkipper": "IPV6_EXT", "TCP": "TCP", "UDP": "UDP", "Payload": "PAYLOAD"}[d]
           for d in cfg["decoders"]]
    p = O.OracleParser(17, dec, outputs=cfg["outputs"])
    reps, t0 = 0, time.perf_counter()
    while True:
        p.decode(data, off, cap, nthreads=threads, layouts=False)
        reps += 1
        el = time.perf_counter() - t0
        if el >= secs:
            return len(off) * reps / el / 1e6, reps, el


def cpu_baseline(head, names, seconds=12.0, batch=262144):
    """the reference's CPU path timed on this box's host
    cores. Go is absent here, so the oracle (oracle/gpk_oracle.c, a bit-exact
    C restatement of the path) stands in ("kind": "port"), one decoder per
    thread over contiguous shards. Bounded samples of each config's workload,
    single-thread and one thread per core of the CPU share. The headline
    config gets `seconds` at full width + a quarter of it single-threaded;
    every other config a quarter and an eighth."""
    threads, nproc, share, model = host_cores()
    out = dict(unit="Mpkts/s", cores=threads, kind="port", nproc=nproc, cpu_share=share, cpu_model=model,
               configs={})
    for name in [head] + [x for x in names if x != head]:
        cfg = CONFIGS[name]
        if cfg.get("strong") or name in ("c3h",) or "x" in name[2:]:
            continue
        full = name == head
        data, off, cap = host_sample(name, batch)
        rT, reps, el = oracle_rate(name, data, off, cap, threads, seconds if full else seconds / 4)
        m = batch // 16
        d1 = data[:int(off[m - 1]) + int(cap[m - 1]) + 16]
        r1, reps1, el1 = oracle_rate(name, d1, off[:m], cap[:m], 1, seconds / 4 if full else seconds / 8)
        mean = float(cap.mean()) + INDEX_BYTES
        row = dict(value=round(rT, 3), threads=threads, single_thread=round(r1, 3),
                   GBps=round(rT * mean / 1e3, 3), single_thread_GBps=round(r1 * mean / 1e3, 3),
                   sample="%d x %d-packet %s sample (%.1f MB) replayed for %.1f s at %d threads; %d x %d packets "
                          "for %.1f s on 1 thread" % (reps, batch, name.upper(), len(data) / 1e6, el, threads,
                                                      reps1, m, el1))
        out["configs"][name] = row
    h = out["configs"][head]
    out.update(value=h["value"], single_thread=h["single_thread"],
               sample="headline %s: %s; oracle/gpk_oracle.c, Go absent on the box (configs: every BASELINE "
                      "config, same method)" % (head.upper(), h["sample"]))
    return out


def pcie_inclusive(name, ctx, n=4 * 2**20, reps=5):
    """gpk_decode_batch_host over a pinned host batch: HtoD copy of bytes and
    index, decode, DtoH copy of the results, synchronous. The rate a host
    source (pcap reader, AF_PACKET ring) sees; never the headline value."""
    import ctypes
    from gopacket_amd import _lib, engine
    cfg = CONFIGS[name]
    L, S = _lib.lib(), _lib.synth_lib()
    kinds = [engine.DECODER_KINDS[d] for d in cfg["decoders"]]
    parser = engine.ParserConfig(17, kinds, outputs=cfg["outputs"])
    nbytes = S.gpk_synth_batch_host(cfg["synth"], 0, n, None, None, None)
    bufs = []

    def pinned(sz):
        p = ctypes.c_void_p()
        _lib.check(L.gpk_host_alloc(ctypes.byref(p), sz))
        bufs.append(p)
        return p.value

    data, off, cap = pinned(nbytes + 16), pinned(8 * n), pinned(4 * n)
    rec, err, fl = pinned(16 * n), pinned(8 * n), pinned(24 * n)
    S.gpk_synth_batch_host(cfg["synth"], 0, n, data, off, cap)
    b = _lib.Batch(data, off, cap, n, nbytes)
    r = _lib.Results(rec, err, fl if cfg["outputs"] & 4 else None, None)
    _lib.check(L.gpk_decode_batch_host(ctx.h, parser.h, ctypes.byref(b), ctypes.byref(r)))
    t0 = time.perf_counter()
    for _ in range(reps):
        _lib.check(L.gpk_decode_batch_host(ctx.h, parser.h, ctypes.byref(b), ctypes.byref(r)))
    el = (time.perf_counter() - t0) / reps
    for p in bufs:
        L.gpk_host_free(p)
    return dict(value=round(n / el / 1e6, 2), unit="Mpkts/s", GBps=round((nbytes + 12 * n) / el / 1e9, 2),
                packets=n, note="gpk_decode_batch_host from pinned memory: HtoD + decode + DtoH")


def c5_cpu(path, threads, nbytes=256 << 20):
    """C5's CPU baseline: NgReader semantics + DecodeLayers
    on the host, over the file's first `nbytes` (a bounded sample, page
    cached): the record walk (gpk_capreader_index_all, the C++ restatement of
    ngread.go:494-718) alone, and walk + the oracle's decode, at 1 thread and
    one per core of the CPU share."""
    import ctypes
    from gopacket_amd import _lib
    from oracle import oracle as O
    L = _lib.lib()
    with open(path, "rb") as f:
        buf = np.frombuffer(f.read(nbytes), np.uint8)
    dec = ["ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP", "PAYLOAD"]
    out = {}
    for t in (1, threads):
        walk = []
        for _ in range(3):
            h = ctypes.c_void_p()
            _lib.check(L.gpk_capreader_create(ctypes.byref(h), 2, 0))  # GPK_CAP_PCAPNG
            x, used = _lib.CapIndex(), ctypes.c_uint64()
            t0 = time.perf_counter()
            rc = L.gpk_capreader_index_all(h, buf.ctypes.data, len(buf), 0, t, ctypes.byref(x), ctypes.byref(used))
            if rc < 0 or not x.n:
                raise RuntimeError("c5_cpu: gpk_capreader_index_all returned %d with %d packets" % (rc, x.n))
            walk.append(time.perf_counter() - t0)
            n = x.n
            off = _lib.host_view(x.offsets, n, np.uint64).copy()
            cap = _lib.host_view(x.caplens, n, np.uint32).copy()
            L.gpk_capindex_free(ctypes.byref(x))
            L.gpk_capreader_destroy(h)
        w = min(walk)
        p = O.OracleParser(17, dec)
        t0 = time.perf_counter()
        p.decode(buf, off, cap, nthreads=t, layouts=False)
        d = time.perf_counter() - t0
        out["threads_%d" % t] = dict(walk_Mpkts_s=round(n / w / 1e6, 2), walk_decode_Mpkts_s=round(n / (w + d) / 1e6, 2),
                                     walk_decode_GBps=round(len(buf) / (w + d) / 1e9, 3))
    out["sample"] = "first %d MiB of the C5 file (%d packets), page cached; walk = gpk_capreader_index_all, " \
                    "decode = oracle/gpk_oracle.c" % (nbytes >> 20, n)
    return out


def htod_probe(total_bytes, slot_bytes=256 << 20, streams=4, reps=2):
    """The host link's rate for C5's copy pattern, in the same run: pinned
    slots of the replay's size -> device, one stream per slot, `streams`
    copies in flight, `total_bytes` per round (the file's size); GB/s of the
    best round, and the same with a single stream."""
    import torch
    hosts = [torch.ones(slot_bytes, dtype=torch.uint8).pin_memory() for _ in range(streams)]
    devs = [torch.empty(slot_bytes, dtype=torch.uint8, device="cuda") for _ in range(streams)]
    sts = [torch.cuda.Stream() for _ in range(streams)]
    nslots = max(1, int(total_bytes // slot_bytes))

    def run(k_streams):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(nslots):
            k = i % k_streams
            with torch.cuda.stream(sts[k]):
                devs[k].copy_(hosts[k], non_blocking=True)
        torch.cuda.synchronize()
        return nslots * slot_bytes / (time.perf_counter() - t0) / 1e9

    run(streams)  # warm
    multi = max(run(streams) for _ in range(reps))
    single = max(run(1) for _ in range(reps))
    del hosts, devs
    return dict(htod_probe_GBps=round(multi, 2), htod_probe_1stream_GBps=round(single, 2),
                htod_pattern="%d x %d MiB pinned slots, %d streams, %.1f GB per round" % (
                    streams, slot_bytes >> 20, streams, nslots * slot_bytes / 1e9))


def c5_replay(ctx, gib=10.0, reps=2, threads=8, cpu_threads=16):
    """BASELINE config C5: a pcapng of the C4 IMIX mix (~gib GiB, written once
    to $TMPDIR, in the page cache) replayed end to end by gpk_replay_file:
    file -> pinned staging slots -> record walk -> HtoD -> decode -> DtoH ->
    per-launch result callback (which counts valid checksums, as a consumer
    would touch the results). Sampled packets are checked against the oracle.
    8 pread threads per slot (the library's default): on the box's 16-CPU share
    they beat 12, 16 and 24 in alternating calls (profiles/r14_c5_threads.txt)."""
    from gopacket_amd import _lib, engine, synth
    from oracle import oracle as O
    S = _lib.synth_lib()
    cfg = CONFIGS["c4"]
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    per = S.gpk_synth_bytes(4, 0, 1 << 20) / (1 << 20) + 32 + 1.5  # frame + EPB header/trailer + padding
    n = int(gib * 2**30 / per)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gpk_c5_%d.pcapng" % os.getpid())
    t0 = time.perf_counter()
    size = S.gpk_synth_write_pcapng(path.encode(), 4, 0, n, cpu_threads)
    if size:
        # the file is replayed from the page cache as a capture written earlier would be: its
        # writeback done first (the first replay otherwise shares the host with the kernel
        # flushing 10 GB of dirty pages: profiles/r15_c5_cold.txt)
        fd = os.open(path, os.O_RDONLY)
        os.fsync(fd)
        os.close(fd)
    gen_s = time.perf_counter() - t0
    if not size:
        raise RuntimeError("could not write %s" % path)
    rng = np.random.default_rng(5)
    sample = sorted(set(int(x) for x in rng.integers(0, n, 2048)) | {0, n - 1})
    picked = {}
    valid = [0]

    def on_batch(first, k, rec, err, fl, ci, cap):
        valid[0] += int(np.count_nonzero(rec["status"] & _lib.ST_L4_VALID))
        lo, hi = np.searchsorted(sample, first), np.searchsorted(sample, first + k)
        for i in sample[lo:hi]:
            j = i - first
            picked[i] = (rec[j].copy(), fl[[j, k + j, 2 * k + j]].copy())

    def replay(p):  # reps calls with parser p; the fastest, and what it delivered for the sample
        rs = []
        for _ in range(reps):
            picked.clear()
            valid[0] = 0
            _, r = ctx.replay_file(p, path, collect=False, on_batch=on_batch, read_threads=threads)
            rs.append(r)
        return rs, dict(picked)

    def check(st, got_pk, decoders, outputs):  # the sample against the oracle with the same parser
        idx = sorted(got_pk)
        pk = [synth.packet(4, i) for i in idx]
        cap = np.array([len(x) for x in pk], np.uint32)
        off = np.concatenate([[0], np.cumsum(cap[:-1], dtype=np.uint64)]).astype(np.uint64)
        ref = O.OracleParser(17, decoders, outputs=outputs).decode(
            np.frombuffer(b"".join(pk) + bytes(16), np.uint8), off, cap, layouts=False)
        got = np.array([got_pk[i][0] for i in idx], _lib.RECORD_DTYPE)
        ok = (st["packets"] == n and st["error"] == "EOF" and len(idx) == len(sample)
              and np.array_equal(got, ref["records"]))
        if ok and outputs & 4:
            gfl = np.stack([got_pk[i][1] for i in idx], axis=1).reshape(-1)
            ok = np.array_equal(gfl, ref["flows"])
        return "%s (%d sampled packets vs oracle)" % ("bit-exact" if ok else "MISMATCH", len(idx))

    fpicked = {}

    def on_batch_fields(first, k, rec, err, fl, ci, cap, fields):
        lo, hi = np.searchsorted(sample, first), np.searchsorted(sample, first + k)
        for i in sample[lo:hi]:
            fpicked[i] = fields[i - first:i - first + 1].copy()

    def replay_fields(p):  # the fused decode + layer fields per launch (gpk_replay_opts.fields_cb)
        rs = []
        for _ in range(reps):
            fpicked.clear()
            _, r = ctx.replay_file(p, path, collect=False, on_batch=on_batch_fields, read_threads=threads,
                                   fields=True)
            rs.append(r)
        return rs, dict(fpicked)

    def check_fields(st, got_f):  # the sampled packets' fields against the oracle's extraction
        idx = sorted(got_f)
        pk = [synth.packet(4, i) for i in idx]
        cap = np.array([len(x) for x in pk], np.uint32)
        off = np.concatenate([[0], np.cumsum(cap[:-1], dtype=np.uint64)]).astype(np.uint64)
        data = np.frombuffer(b"".join(pk) + bytes(16), np.uint8)
        ref = O.OracleParser(17, ["ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP", "PAYLOAD"],
                             outputs=7).decode(data, off, cap, layouts=True)
        want = O.extract_fields(data, off, ref["layouts"])
        got = np.stack([got_f[i].view(np.uint8).reshape(-1) for i in idx])
        ok = st["packets"] == n and len(idx) == len(sample) and np.array_equal(got, want)
        return "%s (%d sampled packets' fields vs oracle)" % ("bit-exact" if ok else "MISMATCH", len(idx))

    seen_bytes = [0]

    def on_batch_packets(first, k, rec, err, fl, ci, cap, pk):
        seen_bytes[0] += int(pk[2].sum(dtype=np.uint64))  # the packets' bytes, handed out in place

    def replay_packets(p):  # gpk_replay_opts.packets_cb: the packets' staging bytes with each launch's results
        rs = []
        for _ in range(reps):
            seen_bytes[0] = 0
            _, r = ctx.replay_file(p, path, collect=False, on_batch=on_batch_packets, read_threads=threads,
                                   packets=True)
            rs.append(r)
        return rs

    cpu = None
    c1 = None
    try:
        runs, got4 = replay(parser)
        valid4 = valid[0]
        runsf, gotf = replay_fields(parser)
        runsp = replay_packets(parser)
        # the same file through C1's parser (Ethernet/IPv4/TCP/Payload, IPv4+TCP checksums): the
        # small-packet dword-aligned kernel on replay batches
        c1cfg = CONFIGS["c1"]
        p1 = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in c1cfg["decoders"]], outputs=c1cfg["outputs"])
        runs1, got1 = replay(p1)
        cpu = c5_cpu(path, cpu_threads)
    finally:
        os.unlink(path)
    probe = htod_probe(size)
    st = min(runs, key=lambda x: x["wall_s"])
    parity = check(st, got4, ["ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP", "PAYLOAD"], 7)
    st1 = min(runs1, key=lambda x: x["wall_s"])
    c1 = dict(parser="Ethernet+IPv4+TCP+Payload, IPv4+TCP checksums (C1's)",
              value=round(st1["packets"] / st1["wall_s"] / 1e6, 2), unit="Mpkts/s",
              GBps=round(st1["file_bytes"] / st1["wall_s"] / 1e9, 2), wall_s=round(st1["wall_s"], 4),
              runs_wall_s=[round(r["wall_s"], 4) for r in runs1], kernel=st1["kernel"],
              kernel_s=round(st1["kernel_s"], 4),
              parity=check(st1, got1, ["ETHERNET", "IPV4", "TCP", "PAYLOAD"], c1cfg["outputs"]))
    stf = min(runsf, key=lambda x: x["wall_s"])
    fields = dict(what="the same replay with gpk_replay_opts.fields_cb: every launch the fused decode + layer "
                       "fields, 128 more bytes per packet copied back",
                  value=round(stf["packets"] / stf["wall_s"] / 1e6, 2), unit="Mpkts/s",
                  GBps=round(stf["file_bytes"] / stf["wall_s"] / 1e9, 2), wall_s=round(stf["wall_s"], 4),
                  runs_wall_s=[round(r["wall_s"], 4) for r in runsf], kernel=stf["kernel"],
                  kernel_s=round(stf["kernel_s"], 4), parity=check_fields(stf, gotf))
    stp = min(runsp, key=lambda x: x["wall_s"])
    packets_row = dict(what="the same replay with gpk_replay_opts.packets_cb: each launch's packets handed out in "
                            "their staging bytes with its results (a staging slot is refilled only after its "
                            "packets were delivered)",
                       value=round(stp["packets"] / stp["wall_s"] / 1e6, 2), unit="Mpkts/s",
                       GBps=round(stp["file_bytes"] / stp["wall_s"] / 1e9, 2), wall_s=round(stp["wall_s"], 4),
                       runs_wall_s=[round(r["wall_s"], 4) for r in runsp],
                       packets_ok=stp["packets"] == n and seen_bytes[0] == stp["packet_bytes"])
    w = st["wall_s"]
    w0 = runs[0]["wall_s"]
    return dict(workload="C5: pcapng replay of the C4 IMIX mix, end to end incl. HtoD/DtoH",
                packets=st["packets"], file_bytes=st["file_bytes"], value=round(st["packets"] / w / 1e6, 2),
                unit="Mpkts/s", GBps=round(st["file_bytes"] / w / 1e9, 2), wall_s=round(w, 4),
                runs_wall_s=[round(r["wall_s"], 4) for r in runs],
                first_call=dict(value=round(st["packets"] / w0 / 1e6, 2), wall_s=round(w0, 4),
                                frac_of_best=round(w / w0, 4), alloc_wait_s=round(runs[0]["alloc_wait_s"], 4),
                                note="allocates and pins the staging buffers (in the background, behind the "
                                     "first reads), which the context keeps for later calls"),
                breakdown_s=dict(read=round(st["read_s"], 4), index=round(st["index_s"], 4),
                                 gpu_copy_decode=round(st["gpu_s"], 4), kernel=round(st["kernel_s"], 4),
                                 deliver=round(st["deliver_s"], 4)),
                batches=st["batches"], slots=st["slots"], l4_valid=valid4, write_s=round(gen_s, 2),
                kernel=st["kernel"], **probe,
                frac_of_htod_probe=round(st["file_bytes"] / w / 1e9 / probe["htod_probe_GBps"], 4),
                parity=parity, c1_parser=c1, fields=fields, packets_cb=packets_row,
                source="page-cached file in %s" % os.path.dirname(path), cpu_baseline=cpu)


def afpacket_pump(ctx, packets=16 * 2**20, block_mib=4, blocks=64, reps=2, batch=1 << 18, cfg_name="c4"):
    """Row (f)2: a TPACKET_V3 ring (blocks x block_mib MiB, laid out as the
    kernel fills it, C4 IMIX packets) drained by gpk_tpacket_pump: ring walk ->
    HtoD of each retired block into the HBM mirror -> decode -> DtoH, blocks
    handed back once on the device. The kernel side is emulated by a thread
    that re-arms every released block at once (a producer that never makes the
    consumer wait), so the figure is the consumer's ceiling. Sampled packets
    are checked against the oracle. cfg_name picks the parser (C4's by
    default; "c1" for C1's Ethernet/IPv4/TCP parser on the same ring)."""
    from gopacket_amd import _lib, afpacket, engine, synth
    from oracle import oracle as O
    S = _lib.synth_lib()
    cfg = CONFIGS[cfg_name]
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    bs = block_mib << 20
    ring = np.zeros(bs * blocks, np.uint8)
    counts = np.zeros(blocks, np.uint64)
    n_ring = int(S.gpk_synth_tpacket_v3(ring.ctypes.data, bs, blocks, 4, 0, 2, 0, counts.ctypes.data))
    rng = np.random.default_rng(6)
    sample = sorted(set(int(x) for x in rng.integers(0, packets, 2048)) | {0, packets - 1})
    picked = {}

    def on_batch(first, k, rec, err, fl, ci, cap):
        lo, hi = np.searchsorted(sample, first), np.searchsorted(sample, first + k)
        for i in sample[lo:hi]:
            j = i - first
            picked[i] = (rec[j].copy(), fl[[j, k + j, 2 * k + j]].copy())

    runs = []
    for _ in range(reps):  # each run: a fresh reader on a ring whose blocks are all handed over
        picked.clear()
        ring[8::bs] = 1
        tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, afpacket.OptFrameSize(4096),
                                 afpacket.OptBlockSize(bs), afpacket.OptNumBlocks(blocks),
                                 afpacket.OptPollTimeout(10_000_000_000))
        prod = S.gpk_synth_tp_producer_start(ring.ctypes.data, bs, blocks)
        try:
            _, st = tp.Pump(ctx, parser, batch_pkts=batch, max_packets=packets, wait=True, inflight=4,
                            collect=False, on_batch=on_batch)
        finally:
            S.gpk_synth_tp_producer_stop(prod)
            tp.Close()
        runs.append(st)
    st = min(runs, key=lambda x: x["wall_s"])
    # packet k of the pump is ring packet k mod n_ring, i.e. synth packet k mod n_ring
    idx = sorted(picked)
    pk = [synth.packet(4, i % n_ring) for i in idx]
    cap = np.array([len(x) for x in pk], np.uint32)
    off = np.concatenate([[0], np.cumsum(cap[:-1], dtype=np.uint64)]).astype(np.uint64)
    ref = O.OracleParser(17, [ORACLE_DEC[d] for d in cfg["decoders"]], outputs=cfg["outputs"]).decode(
        np.frombuffer(b"".join(pk) + bytes(16), np.uint8), off, cap, layouts=False)
    got = np.array([picked[i][0] for i in idx], _lib.RECORD_DTYPE)
    gfl = np.stack([picked[i][1] for i in idx], axis=1).reshape(-1)
    ok = (st["packets"] == packets and len(idx) == len(sample) and np.array_equal(got, ref["records"])
          and (not cfg["outputs"] & 4 or np.array_equal(gfl, ref["flows"])))
    w = st["wall_s"]
    return dict(workload="(f)2: AF_PACKET TPACKET_V3 ring -> HBM -> decode (C4 IMIX mix), emulated kernel producer",
                parser=" ".join(cfg["decoders"]), kernel=st.get("kernel"),
                ring="%d x %d MiB blocks, %d packets per lap" % (blocks, block_mib, n_ring),
                packets=st["packets"], value=round(st["packets"] / w / 1e6, 2), unit="Mpkts/s",
                packet_GBps=round(st["packet_bytes"] / w / 1e9, 2),
                ring_GBps=round(st["ring_bytes_copied"] / w / 1e9, 2), wall_s=round(w, 4),
                runs_wall_s=[round(r["wall_s"], 4) for r in runs],
                breakdown_s=dict(index=round(st["index_s"], 4), gpu_copy_decode=round(st["gpu_s"], 4),
                                 kernel=round(st["kernel_s"], 4)),
                batches=st["batches"], batch_pkts=batch, waits=st["waits"],
                parity="%s (%d sampled packets vs oracle)" % ("bit-exact" if ok else "MISMATCH", len(idx)))


def flow_grouping(ctx, n=64 * 2**20, reps=5):
    """Row (f)3: C6 traffic (C4's frames, endpoints from a heavy-tailed pool of
    2^20 flows in both directions, 5 % IPv4 fragments) generated in HBM,
    decoded with layouts, then grouped on the device by each consumer's key
    (gpk_group_batch). Timed with HIP events on the stream. Sampled groups are
    checked against the oracle's key of their packets."""
    import torch
    from gopacket_amd import _lib, engine, flows, synth
    from oracle import flows_oracle as FO
    from oracle import oracle as O
    dec = ["ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP", "PAYLOAD"]
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in CONFIGS["c4"]["decoders"]], outputs=7)
    stream = torch.cuda.current_stream()
    d, o, c = synth.device_batch(6, 0, n)
    rec = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
    fl = torch.zeros(3 * n, dtype=torch.int64, device="cuda")
    lay = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ctx.decode_device(parser, d, o, c, rec, err, fl, lay, stream=stream)
    e0.record(stream)
    for _ in range(reps):
        ctx.decode_device(parser, d, o, c, rec, err, fl, lay, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    dec_ms = e0.elapsed_time(e1) / reps
    g = flows.Grouper(n)
    out = {}
    for name, kind, buckets in (("connection", FO.CONNECTION, 8), ("defrag", FO.DEFRAG, 8),
                                ("net_bucket8", FO.NET_BUCKET, 8)):
        res = g.group(d, o, c, rec, lay, fl, kind=kind, buckets=buckets)  # warm
        e0.record(stream)
        for _ in range(reps):
            res = g.group(d, o, c, rec, lay, fl, kind=kind, buckets=buckets)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        G, K = res["counts"].cpu().tolist()
        ok = True
        if kind != FO.NET_BUCKET:  # sampled groups: one oracle key per group, distinct across groups
            perm = res["perm"][:K].cpu().numpy()
            start = res["start"][:G + 1].cpu().numpy()
            rng = np.random.default_rng(4)
            keys = []
            for gg in rng.choice(G, min(G, 64), replace=False):
                idx = perm[start[gg]:start[gg + 1]][:32]
                pk = [synth.packet(6, int(i)) for i in idx]
                cap = np.array([len(x) for x in pk], np.uint32)
                off = np.concatenate([[0], np.cumsum(cap[:-1], dtype=np.uint64)]).astype(np.uint64)
                r = O.OracleParser(17, dec).decode(np.frombuffer(b"".join(pk) + bytes(16), np.uint8), off, cap)
                ks = {FO.packet_key(kind, p, r["records"][k], r["layouts"][k], 0, 8) for k, p in enumerate(pk)}
                ok = ok and len(ks) == 1 and not isinstance(next(iter(ks)), int)
                keys.append(next(iter(ks)))
            ok = ok and len(set(keys)) == len(keys)
        out[name] = dict(ms=round(ms, 4), Mpkts_s=round(n / ms / 1e3, 1), groups=G, keyed_packets=K,
                         parity="%s (sampled groups vs oracle keys)" % ("ok" if ok else "MISMATCH")
                         if kind != FO.NET_BUCKET else "see tests/test_flows_gpu.py")
    # fused: the decode kernel derives the key (no layouts, no second header pass)
    fused = {}
    for name, kind in (("connection", FO.CONNECTION), ("defrag", FO.DEFRAG)):
        res = g.decode_group(ctx, parser, d, o, c, rec, err, fl, kind=kind)
        e0.record(stream)
        for _ in range(reps):
            res = g.decode_group(ctx, parser, d, o, c, rec, err, fl, kind=kind)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        G, K = res["counts"].cpu().tolist()
        same = (G, K) == (out[name]["groups"], out[name]["keyed_packets"])
        fused[name] = dict(decode_and_group_ms=round(ms, 4), Mpkts_s=round(n / ms / 1e3, 1),
                           separate_ms=round(dec_ms + out[name]["ms"], 4),
                           same_groups_as_separate="yes" if same else "NO")
    out["fused_decode_group"] = fused
    g.close()
    del d, o, c, rec, err, fl, lay
    torch.cuda.empty_cache()
    # CPU baseline: the reference keys each packet with one map lookup (single
    # goroutine per StreamPool / defragmenter); its C restatement with a hash
    # map, one thread, over a 1 Mi-packet host sample of the same traffic
    # (decode results precomputed, untimed)
    m = 1 << 20
    hd, ho, hc = synth.host_batch(6, 0, m)
    hr = O.OracleParser(17, dec).decode(hd, ho, hc, nthreads=16, layouts=True)
    cpu = {}
    for name, kind in (("connection", FO.CONNECTION), ("defrag", FO.DEFRAG), ("net_bucket8", FO.NET_BUCKET)):
        reps, t0 = 0, time.perf_counter()
        while True:
            O.group_batch(kind, hd, ho, hr["records"], hr["layouts"], hr["flows"], 8)
            reps += 1
            el = time.perf_counter() - t0
            if el >= 2.0:
                break
        cpu[name] = round(reps * m / el / 1e6, 2)
    return dict(workload="(f)3: C6 64M packets (IMIX, 2^20 heavy-tailed flows, both directions, 5%% IPv4 "
                         "fragments), decode with layouts, then group by consumer key in HBM",
                packets=n, decode_with_layouts_ms=round(dec_ms, 4), grouping=out,
                cpu_baseline=dict(Mpkts_s=cpu, cores=1, kind="port",
                                  sample="1 Mi C6 packets, oracle/flows_oracle.c (one hash-map lookup per packet)"))


def bpf_filter_bench(ctx, n=64 * 2**20, reps=10):
    """Row (f)4: classic BPF (the reference's own TestBPFInstruction programs)
    over 64M C4 IMIX packets in HBM: gpk_bpf_run (return value per packet) and
    gpk_bpf_select (compacted matching index). Timed with HIP events; a
    sample of 2048 packets checked against the oracle (libpcap bpf_filter)."""
    import torch
    from gopacket_amd import bpf, synth
    from oracle import oracle as O
    d, o, c = synth.device_batch(4, 0, n)
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "bpf_programs.json")))
    progs = {x["filter"]: x["insns"] for x in g["instruction_cases"] if not x["error"]}
    rng = np.random.default_rng(8)
    sample = np.unique(rng.integers(0, n, 2048))
    out = {}
    ret = torch.empty(n, dtype=torch.int32, device="cuda")
    for name, prog in progs.items():
        f = bpf.NewBPFInstructionFilter(prog)
        f.Run(d, o, c, ret=ret)
        e0.record(stream)
        for _ in range(reps):
            f.Run(d, o, c, ret=ret)
        e1.record(stream)
        torch.cuda.synchronize()
        run_ms = e0.elapsed_time(e1) / reps
        f.Select(d, o, c)
        e0.record(stream)
        for _ in range(reps):
            oo, oc, oi, cnt = f.Select(d, o, c)
        e1.record(stream)
        torch.cuda.synchronize()
        sel_ms = e0.elapsed_time(e1) / reps
        got = ret.cpu().numpy()[sample].astype(np.uint32)
        pk = [synth.packet(4, int(i)) for i in sample]
        cap = np.array([len(x) for x in pk], np.uint32)
        off = np.concatenate([[0], np.cumsum(cap[:-1], dtype=np.uint64)]).astype(np.uint64)
        ref = O.bpf_batch(prog, np.frombuffer(b"".join(pk) + bytes(16), np.uint8), off, cap)
        out[name] = dict(insns=len(prog), run_ms=round(run_ms, 4), run_Gpkts_s=round(n / run_ms / 1e6, 2),
                         select_ms=round(sel_ms, 4), matches=int(cnt.item()),
                         index_GBps=round(n * 16 / (run_ms * 1e-3) / 1e9, 1),
                         parity="%s (%d sampled packets vs oracle)" % ("bit-exact" if np.array_equal(got, ref)
                                                                       else "MISMATCH", len(sample)))
        f.close()
    # CPU baseline: libpcap's bpf_filter restated (oracle/bpf_oracle.c), one
    # thread as pcap_offline_filter runs per handle, over a 1 Mi-packet sample
    m = 1 << 20
    hd, ho, hc = synth.host_batch(4, 0, m)
    for name, prog in progs.items():
        reps, t0 = 0, time.perf_counter()
        while True:
            O.bpf_batch(prog, hd, ho, hc)
            reps += 1
            el = time.perf_counter() - t0
            if el >= 1.5:
                break
        out[name]["cpu_baseline"] = dict(Mpkts_s=round(reps * m / el / 1e6, 2), cores=1, kind="port",
                                         sample="1 Mi C4 packets, oracle/bpf_oracle.c")
    return dict(workload="(f)4: classic BPF (pcap_test.go TestBPFInstruction programs) over 64M C4 IMIX "
                         "packets in HBM", packets=n, programs=out)


def fields_bench(ctx, name="c4", n=64 * 2**20, reps=5, check_packets=4 << 20, first=0, threads=None):
    """Layer fields with the decode (gpk_decode_batch_fields, no layouts: ONE
    launch that also writes each packet's 128-byte gpk_fields record) against
    the two-launch form (decode with layouts, then gpk_extract_fields), on the
    64M C4 batch in HBM; HIP events on the launch stream, median of reps.
    frac counts the algorithmic read bytes (caplen + 12) like the decode rows;
    written bytes per packet are reported beside it. The first check_packets
    packets of the fused run are compared with the oracle (records, error
    arguments, flows, fields)."""
    import torch
    from gopacket_amd import _lib, engine, synth
    from oracle import oracle as O
    cfg = CONFIGS[name]
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    stream = torch.cuda.current_stream()
    data, off, cap = synth.device_batch(cfg["synth"], first, n, stream=stream)
    rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
    fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
    fields = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    lay = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    payload = int(cap.sum(dtype=torch.int64).item())
    algo = payload + INDEX_BYTES * n

    def timed(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ts = []
        for k in range(reps + 2):
            ev[0].record(stream)
            fn()
            ev[1].record(stream)
            torch.cuda.synchronize()
            if k >= 2:
                ts.append(ev[0].elapsed_time(ev[1]))
        return sorted(ts)[len(ts) // 2]

    two = timed(lambda: (ctx.decode_device(parser, data, off, cap, rec, err, fl, lay, stream=stream),
                         ctx.extract_fields(data, off, cap, lay, fields, stream=stream)))
    fused = timed(lambda: ctx.decode_device_fields(parser, data, off, cap, rec, err, fl, fields, stream=stream))
    # parity of the fused run (the last launch wrote every output)
    dec = [ORACLE_DEC[d] for d in cfg["decoders"]]
    p = O.OracleParser(17, dec, outputs=cfg["outputs"])
    bad = 0
    chunk = 1 << 20
    for a in range(0, min(n, check_packets), chunk):
        b = min(n, a + chunk)
        o = off[a:b].cpu().numpy().astype(np.uint64)
        c = cap[a:b].cpu().numpy().astype(np.uint32)
        lo, hi = int(o.min()), int((o + c).max())
        host = np.zeros(hi - lo + 16, np.uint8)
        host[:hi - lo] = data[lo:hi].cpu().numpy()
        ref = p.decode(host, o - np.uint64(lo), c, nthreads=threads or rank_threads(), layouts=True)
        ok = rec[a * 16:b * 16].cpu().numpy().view(_lib.RECORD_DTYPE) == ref["records"]
        ok &= (err[2 * a:2 * b].cpu().numpy().view(np.uint32).reshape(-1, 2) == ref["err_args"].reshape(-1, 2)).all(1)
        rf = ref["flows"].reshape(3, -1)
        for k in range(3):
            ok &= fl[k * n + a:k * n + b].cpu().numpy().view(np.uint64) == rf[k]
        want = O.extract_fields(host, o - np.uint64(lo), ref["layouts"])
        ok &= (fields[a * 128:b * 128].cpu().numpy().reshape(-1, 128) == want).all(1)
        bad += int((~ok).sum())
    written = 16 + 24 + 128  # record, three flow hashes, fields (+8 on error)
    skel = skeleton_ms(cfg, data, off, cap, n, 5, stream, wbytes=written)
    ach = algo / (fused * 1e-3) / 1e9
    traffic, traffic_profile = load_traffic("c4f", n)  # the fused launch's PMC profile (tools/profile.sh c4f)
    res = dict(workload=CONFIGS[name]["workload"] + " + layer fields (gpk_decode_batch_fields)",
               kernel=ctx.kernel_name(parser, data, off, cap, layouts=_lib.NAME_FIELDS),
               blocks_per_cu=ctx.occupancy(parser, data, off, cap, layouts=_lib.NAME_FIELDS),
               kernel_ms=round(fused, 4), value=round(n / fused / 1e3, 2), unit="Mpkts/s",
               achieved_GBps=round(ach, 1), frac=round(ach / HBM_PEAK_GBS, 4),
               written_bytes_per_packet=written, traffic=traffic, traffic_profile=traffic_profile,
               read_plus_written_GBps=round((algo + written * n) / (fused * 1e-3) / 1e9, 1),
               skeleton_ms=round(skel, 4), of_skeleton=round(skel / fused, 4),
               two_launch_ms=round(two, 4), two_launch_kernels=[ctx.kernel_name(parser, data, off, cap, layouts=True),
                                                                "fields_kernel"],
               parity=("bit-exact" if not bad else "MISMATCH (%d packets)" % bad) +
               " (first %d packets vs oracle: records, error arguments, flows, fields)" % min(n, check_packets))
    del data, off, cap, rec, err, fl, fields, lay
    torch.cuda.empty_cache()
    return res


def load_traffic(name, n):
    """HBM bytes per launch of the decode kernel from the committed PMC
    profile (profiles/hbm_traffic.json, tools/make_profiles.py): measured
    bytes per packet x packets per launch, and the profile's tag. (None,
    None) if not profiled."""
    path = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    try:
        t = json.load(open(path))[name]
        return (round((t["fetch_bytes_per_packet"] + t["write_bytes_per_packet"]) * n),
                "profiles/%s_pmc.json (%s)" % (t["profile"], t.get("kernel", "decode_kernel")))
    except (OSError, KeyError, ValueError):
        return None, None


def c5_sharded(ctx, rank, world, gib=10.0, reps=2, threads=8):
    """C5 at N GPUs: rank 0 writes the same pcapng as c5_replay (the C4 IMIX
    mix, ~gib GiB, page cached); every rank replays its byte range of it
    (shard.replay_file_sharded -> gpk_replay_file_range: its own staging, HtoD
    link, walk and decode, no data exchange; the ranks swap only their range
    outcomes, and an inexact split is redone, so the ranks' results in rank
    order are always the whole file's). The job's wall per repetition is the
    slowest rank's, from a common barrier; value = the file's packets / the best
    repetition's job wall. Each rank checks its sampled packets against the
    oracle at their global index."""
    import torch
    import torch.distributed as dist
    from gopacket_amd import _lib, engine, shard, synth
    from oracle import oracle as O
    S = _lib.synth_lib()
    cfg = CONFIGS["c4"]
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    per = S.gpk_synth_bytes(4, 0, 1 << 20) / (1 << 20) + 32 + 1.5
    n = int(gib * 2**30 / per)
    tag = os.environ.get("MASTER_PORT", str(os.getpid()))
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gpk_c5_shared_%s.pcapng" % tag)
    gen_s, size = 0.0, 0
    if rank == 0:
        t0 = time.perf_counter()
        size = S.gpk_synth_write_pcapng(path.encode(), 4, 0, n, host_cores()[0])
        if size:
            fd = os.open(path, os.O_RDONLY)
            os.fsync(fd)
            os.close(fd)
        gen_s = time.perf_counter() - t0
    ok = gather_obj(rank != 0 or size > 0, world)
    if not all(ok):
        raise RuntimeError("could not write %s" % path)
    rng = np.random.default_rng(5 + rank)
    local_sample = np.unique(rng.integers(0, n // world + n // (4 * world) + 1, 2048 // world + 64))
    picked = {}

    def on_batch(first, k, rec, err, fl, ci, cap):
        lo, hi = np.searchsorted(local_sample, first), np.searchsorted(local_sample, first + k)
        for i in local_sample[lo:hi]:
            j = int(i) - first
            picked[int(i)] = (rec[j].copy(), fl[[j, k + j, 2 * k + j]].copy())

    runs = []
    try:
        for _ in range(reps):
            picked.clear()
            barrier(world)
            t0 = time.perf_counter()
            _, st, info = shard.replay_file_sharded(ctx, parser, path, rank, world, collect=False,
                                                     on_batch=on_batch, read_threads=threads)
            wall = time.perf_counter() - t0
            runs.append((wall, st, info, dict(picked)))
    finally:
        barrier(world)
        if rank == 0:
            os.unlink(path)
    probe = htod_probe(n * per / world)  # every rank's link at once, its share of the file per round
    walls = [gather_obj(r[0], world) for r in runs]
    best = min(range(reps), key=lambda k: max(walls[k]))
    wall, st, info, got = runs[best]
    # this rank's sampled packets against the oracle, at their global index
    idx = sorted(i for i in got if not info["dropped"])
    parity = "no sampled packets"
    if idx:
        pk = [synth.packet(4, info["first_packet"] + i) for i in idx]
        cap = np.array([len(x) for x in pk], np.uint32)
        off = np.concatenate([[0], np.cumsum(cap[:-1], dtype=np.uint64)]).astype(np.uint64)
        ref = O.OracleParser(17, [ORACLE_DEC[d] for d in cfg["decoders"]], outputs=cfg["outputs"]).decode(
            np.frombuffer(b"".join(pk) + bytes(16), np.uint8), off, cap, layouts=False)
        g = np.array([got[i][0] for i in idx], _lib.RECORD_DTYPE)
        gfl = np.stack([got[i][1] for i in idx], axis=1).reshape(-1)
        good = np.array_equal(g, ref["records"]) and np.array_equal(gfl, ref["flows"])
        parity = "%s (%d sampled packets vs oracle)" % ("bit-exact" if good else "MISMATCH", len(idx))
    mine = dict(rank=rank, wall_s=round(wall, 4), packets=int(st["packets"]), first_packet=info["first_packet"],
                file_bytes=int(st.get("file_bytes", 0)), error=st.get("error"), redo=info["redo_rank"] == rank,
                dropped=info["dropped"], range=st.get("range"), parity=parity,
                breakdown_s=dict(read=round(st.get("read_s", 0), 4), index=round(st.get("index_s", 0), 4),
                                 gpu_copy_decode=round(st.get("gpu_s", 0), 4), kernel=round(st.get("kernel_s", 0), 4),
                                 deliver=round(st.get("deliver_s", 0), 4)),
                htod_probe_GBps=probe["htod_probe_GBps"])
    ranks = gather_obj(mine, world)
    total = sum(r["packets"] for r in ranks)
    jw = max(walls[best])
    last = max(r["rank"] for r in ranks if not r["dropped"])
    exact = total == n and ranks[last]["error"] == "EOF" and all(
        r["parity"].startswith("bit-exact") for r in ranks if not r["dropped"])
    return dict(workload="C5 at %d GPUs: one pcapng of the C4 IMIX mix, each rank replays its byte range end to "
                         "end incl. HtoD/DtoH (gpk_replay_file_range)" % world,
                packets=total, file_packets=n, value=round(total / jw / 1e6, 2), unit="Mpkts/s",
                GBps=round(sum(r["file_bytes"] for r in ranks) / jw / 1e9, 2), wall_s=round(jw, 4),
                runs_wall_s=[round(max(w), 4) for w in walls], scaling="strong",
                redo_rank=info["redo_rank"], write_s=round(gen_s, 2),
                htod_probe_GBps_sum=round(sum(r["htod_probe_GBps"] for r in ranks), 2),
                parity=("bit-exact" if exact else "MISMATCH") + " (%d of %d packets delivered across ranks, the "
                       "last rank's reader at EOF, every rank's sample vs oracle)" % (total, n),
                ranks=ranks, source="page-cached file in %s" % os.path.dirname(path))


def narrow_row(r, world, name=None):
    """The config's decode with the 8-byte record (gpk_decode_batch_narrow),
    timed beside the 16-byte one on the same batch: kernel time (the slowest
    rank's), rate by kernel time, HBM fraction of the same algorithmic bytes,
    and the 16-byte kernel's time over it. Its every-packet parity is in the
    config's full_parity."""
    nr = r.get("narrow")
    if not nr:
        return None
    k = nr["kernel_ms"]
    pk = r["strong"]["total_packets"] if r.get("strong") else r["n"] * world
    ach = r["algo_bytes"] / (k * 1e-3) / 1e9
    traffic, profile = load_traffic(name + "n", r["n"]) if name else (None, None)
    return dict(kernel_ms=round(k, 4), value_by_kernel=round(pk / k / 1e3, 2), unit="Mpkts/s",
                achieved_GBps=round(ach, 1), frac=round(ach / HBM_PEAK_GBS, 4),
                speedup_vs_16B=round(r["kernel_ms"] / k, 4), traffic=traffic, traffic_profile=profile,
                record="gpk_record8: 8 B per packet, the full 16 B record in a side array only where it does not "
                       "fit (Correct != the header Checksum, or more than 8 layers)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--packets", type=int, default=64 * 2**20, help="packets per GPU")
    ap.add_argument("--configs", default=None,
                    help="first one is the headline (default c3,c2,c4,c1, plus c4s strong scaling when N > 1)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-full-parity", action="store_true",
                    help="skip the every-packet comparison against the oracle (sampled parity only)")
    ap.add_argument("--no-probe", action="store_true", help="skip the streaming-read reference kernel")
    ap.add_argument("--no-narrow", action="store_true",
                    help="skip the narrow-record timing beside each config (it launches the same kernel symbols: "
                         "keep it out of kernel traces that average by name)")
    ap.add_argument("--pcie", action="store_true", default=True,
                    help="time the host-buffer path too (PCIe-inclusive, N=1; on by default)")
    ap.add_argument("--no-pcie", dest="pcie", action="store_false", help="skip the PCIe-inclusive row")
    ap.add_argument("--c5", type=float, default=10.0, metavar="GIB",
                    help="config C5: replay a GIB-GiB pcapng end to end (gpk_replay_file); 0 = skip")
    ap.add_argument("--afpacket", type=int, default=0, metavar="MPKTS",
                    help="also drain MPKTS Mi packets from an emulated TPACKET_V3 ring (gpk_tpacket_pump)")
    ap.add_argument("--flows", action="store_true",
                    help="also time row (f)3: flow-keyed grouping of 64M C6 packets (gpk_group_batch)")
    ap.add_argument("--bpf", action="store_true", help="also time row (f)4: classic BPF over 64M C4 packets")
    ap.add_argument("--no-fields", action="store_true",
                    help="skip the layer-fields row (64M C4 decode + fields in one launch vs two)")
    ap.add_argument("--tables", default="auto", choices=["auto", "global"],
                    help="next-layer tables: compact LDS copy (auto) or device-memory tables (global)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL (one rank per GPU); gloo + --same-device rehearses ranks on one GPU")
    ap.add_argument("--same-device", action="store_true", help="every rank on cuda:0 (rehearsal only)")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the process group at world size 1 too (barrier / max over ranks through it)")
    args = ap.parse_args()

    mode, cmd = launch_plan(args.gpus, os.environ, sys.argv[1:])
    if mode == "spawn":  # nothing here has touched the GPU
        sys.exit(spawn_ranks(cmd))

    import torch
    import torch.distributed as dist
    rank, world, local = dist_init(args.dist_backend, args.same_device, args.force_dist)
    if world != args.gpus:
        raise SystemExit("bench.py: rank %d sees world size %d, --gpus %d" % (rank, world, args.gpus))
    from gopacket_amd import engine
    ctx = engine.Context(local)
    if args.tables == "global":
        from gopacket_amd import _lib
        ctx.set_table_mode(_lib.TABLES_GLOBAL)
    names = (args.configs or ("c3,c2,c4,c1" + (",c4s" if world > 1 else ""))).split(",")
    results = {}
    for name in names:
        results[name] = run_config(name, args.packets, args.steps, args.warmup, rank, world, ctx,
                                   check_sample=0 if args.no_parity else 2048,
                                   probe=not args.no_probe,
                                   full_check=not (args.no_parity or args.no_full_parity),
                                   narrow=not args.no_narrow)
    threads = host_cores()[0]
    # every rank runs the rows below its own shard at N > 1 (weak: its own 64M batch; C5: its byte range)
    fields_ranks = None
    if not args.no_fields:
        fr = fields_bench(ctx, n=args.packets, first=rank * args.packets, threads=rank_threads())
        fields_ranks = gather_obj(dict(fr, rank=rank), world)
    c5 = None
    if args.c5 > 0:
        c5 = (c5_replay(ctx, gib=args.c5, cpu_threads=threads) if world == 1
              else c5_sharded(ctx, rank, world, gib=args.c5))
    if rank == 0:
        head = names[0]
        r = results[head]
        total_pkts = r["n"] * world * args.steps
        value = total_pkts / r["wall_s"] / 1e6
        achieved = r["algo_bytes"] / (r["kernel_ms"] * 1e-3) / 1e9
        traffic, traffic_profile = load_traffic(head, r["n"])
        out = {
            "metric": "Mpkts/s device-resident Eth/IPv4/TCP decode+cksum+flow-hash; % HBM roofline",
            "value": round(value, 2), "unit": "Mpkts/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(r["wall_s"] / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (deterministic splitmix64 per packet index, generated in HBM)",
            "config": {"workload": CONFIGS[head]["workload"], "packets_per_gpu": r["n"],
                       "payload_bytes_per_gpu": r["payload_bytes"], "parallelism": "shard%d" % world,
                       "parser": "+".join(CONFIGS[head]["decoders"])},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_profile": traffic_profile, "kernel": r["kernel"],
                         "blocks_per_cu": r["blocks_per_cu"],
                         "traffic_unit": "bytes per launch", "kernel_ms": round(r["kernel_ms"], 4),
                         "kernel_ms_ranks": r["kernel_ms_ranks"],
                         "algo_bytes_per_launch": r["algo_bytes"],
                         "probe_read_GBps": r["probe_gbs"] and round(r["probe_gbs"], 1),
                         "skeleton_ms": r["skeleton_ms"] and round(r["skeleton_ms"], 4),
                         "of_skeleton": r["skeleton_ms"] and round(r["skeleton_ms"] / r["kernel_ms"], 4)},
            "parity": r["parity"],
            "full_parity": r["full_parity"],
            "narrow": narrow_row(r, world, head),
            "dist_backend": dist.get_backend() if dist.is_initialized() else None,
            "configs": {},
        }
        for name in names[1:]:
            s = results[name]
            ach = s["algo_bytes"] / (s["kernel_ms"] * 1e-3) / 1e9
            st = s["strong"]
            pk = st["total_packets"] if st else s["n"] * world
            row = {"workload": CONFIGS[name]["workload"],
                   "value": round(pk * args.steps / s["wall_s"] / 1e6, 2), "unit": "Mpkts/s",
                   "kernel": s["kernel"], "blocks_per_cu": s["blocks_per_cu"], "kernel_ms": round(s["kernel_ms"], 4),
                   "kernel_ms_ranks": s["kernel_ms_ranks"], "achieved_GBps": round(ach, 1),
                   "frac": round(ach / HBM_PEAK_GBS, 4), "parity": s["parity"], "full_parity": s["full_parity"],
                   "probe_read_GBps": s["probe_gbs"] and round(s["probe_gbs"], 1),
                   "skeleton_ms": s["skeleton_ms"] and round(s["skeleton_ms"], 4),
                   "of_skeleton": s["skeleton_ms"] and round(s["skeleton_ms"] / s["kernel_ms"], 4),
                   "narrow": narrow_row(s, world, name)}
            if st:
                row.update(scaling="strong", total_packets=st["total_packets"], byte_balance=st["balance"],
                           note="one batch split at byte-balanced cuts; kernel_ms/achieved: the slowest rank's "
                                "shard (kernel_ms_ranks: every rank's)")
            out["configs"][name] = row
        if args.pcie and world == 1:
            out["pcie_inclusive"] = pcie_inclusive(head, ctx)
        if fields_ranks:
            out["fields"] = dict(fields_ranks[0])
            if world > 1:
                out["fields"]["ranks"] = [{k: f[k] for k in ("rank", "value", "kernel_ms", "frac", "parity")}
                                          for f in fields_ranks]
                out["fields"]["value_all_ranks"] = round(sum(f["value"] for f in fields_ranks), 2)
        if c5 is not None:
            out["c5"] = c5
        if args.bpf and world == 1:
            out["bpf"] = bpf_filter_bench(ctx)
        if args.flows and world == 1:
            out["flows"] = flow_grouping(ctx)
        if args.afpacket > 0 and world == 1:
            out["afpacket"] = afpacket_pump(ctx, packets=args.afpacket * 2**20)
            out["afpacket"]["c1_parser"] = afpacket_pump(ctx, packets=args.afpacket * 2**20, cfg_name="c1")
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(head, names, seconds=args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
            if world > 1:
                out["cpu_baseline_note"] = ("measured at N=1 only (BENCH line): at N>1 the ranks share the host "
                                            "cores, which the per-rank parity checks use")
        print(json.dumps(out))
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
