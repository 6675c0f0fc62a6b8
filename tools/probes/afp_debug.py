"""Diagnose the pump bench: which sampled packets differ, pinned vs pageable ring."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from gopacket_amd import _lib, afpacket, engine, synth
from oracle import oracle as O

S = _lib.synth_lib()
ctx = engine.Context(0)
dec = ["ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP", "PAYLOAD"]
parser = engine.ParserConfig(17, [1, 2, 3, 4, 5, 6, 7, 8], outputs=7)
for block_mib, blocks, packets, batch in [(4, 64, 4 << 20, 1 << 18), (4, 64, 4 << 20, 1 << 20), (1, 64, 4 << 20, 1 << 17)]:
    bs = block_mib << 20
    ring = np.zeros(bs * blocks, np.uint8)
    n_ring = int(S.gpk_synth_tpacket_v3(ring.ctypes.data, bs, blocks, 4, 0, 2, 0, None))
    tp = afpacket.AttachRing(ring, 2, afpacket.OptFrameSize(4096), afpacket.OptBlockSize(bs),
                             afpacket.OptNumBlocks(blocks), afpacket.OptPollTimeout(10_000_000_000))
    prod = S.gpk_synth_tp_producer_start(ring.ctypes.data, bs, blocks)
    t = time.time()
    got, st = tp.Pump(ctx, parser, batch_pkts=batch, max_packets=packets, wait=True, inflight=4)
    S.gpk_synth_tp_producer_stop(prod)
    print("cfg", block_mib, blocks, packets, batch, "n_ring", n_ring, {k: st[k] for k in ("packets", "batches", "waits", "wall_s", "index_s", "gpu_s", "ring_bytes_copied")}, time.time() - t)
    idx = np.arange(0, packets, 997)
    pk = [synth.packet(4, int(i) % n_ring) for i in idx]
    cap = np.array([len(x) for x in pk], np.uint32)
    off = np.concatenate([[0], np.cumsum(cap[:-1], dtype=np.uint64)]).astype(np.uint64)
    ref = O.OracleParser(17, dec).decode(np.frombuffer(b"".join(pk) + bytes(16), np.uint8), off, cap, layouts=False)
    bad = np.nonzero(got["records"][idx] != ref["records"])[0]
    capbad = np.nonzero(got["caplens"][idx] != cap)[0]
    print("  record mismatches", len(bad), "of", len(idx), "first", idx[bad[:10]], "caplen mismatches", len(capbad), idx[capbad[:10]])
    if len(bad):
        i = bad[0]
        print("  got", got["records"][idx[i]], "ref", ref["records"][i], "cap", got["caplens"][idx[i]], cap[i])
