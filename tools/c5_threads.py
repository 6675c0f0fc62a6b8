#!/usr/bin/env python3
"""In-process A/B of the C5 replay's pread threads per slot: one 10 GiB C4-mix
pcapng in the page cache, one context (buffers kept), calls alternating over
the thread counts so box drift hits every count alike.

    python tools/c5_threads.py [--gib 10] [--threads 8,12,16,24] [--rounds 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=10.0)
    ap.add_argument("--threads", default="8,12,16,24")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--affinity", default="lib", help="comma list of 'lib' (the library pins its reader "
                    "threads and the calling thread to the GPU's NUMA node), 'lib1' (the reader threads only), 'all' (GPK_REPLAY_NUMA=0: the inherited CPU set) and "
                    "'local' (GPK_REPLAY_NUMA=0, the calling thread on the GPU's node: the reader threads "
                    "inherit it)")
    a = ap.parse_args()
    import torch  # noqa: F401
    from gopacket_amd import _lib, engine
    import bench
    S = _lib.synth_lib()
    cfg = bench.CONFIGS["c4"]
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    per = S.gpk_synth_bytes(4, 0, 1 << 20) / (1 << 20) + 33.5
    n = int(a.gib * 2**30 / per)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gpk_c5t_%d.pcapng" % os.getpid())
    S.gpk_synth_write_pcapng(path.encode(), 4, 0, n, 16)
    counts = [int(x) for x in a.threads.split(",")]
    ctx = engine.Context(0)
    all_cpus = os.sched_getaffinity(0)
    sets = {"all": all_cpus, "lib": all_cpus, "lib1": all_cpus}
    if "local" in a.affinity:
        pr = torch.cuda.get_device_properties(0)
        bdf = "%04x:%02x:%02x.0" % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
        dev = "/sys/bus/pci/devices/" + bdf
        cl = open(dev + "/local_cpulist").read().strip()
        node = open(dev + "/numa_node").read().strip()
        cpus = set()
        for part in cl.split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        sets["local"] = cpus & all_cpus or cpus
        print("GPU %s: NUMA node %s, local CPUs %s (%d of the %d inherited)" % (
            bdf, node, cl, len(sets["local"]), len(all_cpus)), flush=True)
    modes = a.affinity.split(",")
    best = {}
    try:
        ctx.replay_file(parser, path, collect=False, on_batch=lambda *x: None)  # allocate + pin the slots
        for r in range(a.rounds):
            for m in modes:
                os.sched_setaffinity(0, sets[m])
                os.environ["GPK_REPLAY_NUMA"] = {"lib": "2", "lib1": "1"}.get(m, "0")
                for t in counts:
                    _, st = ctx.replay_file(parser, path, collect=False, on_batch=lambda *x: None, read_threads=t)
                    gbs = st["file_bytes"] / st["wall_s"] / 1e9
                    best[m, t] = max(best.get((m, t), 0.0), gbs)
                    print("round %d %s threads %2d: %.4f s, %.2f GB/s, read %.3f index %.3f gpu %.3f" % (
                        r, m, t, st["wall_s"], gbs, st["read_s"], st["index_s"], st["gpu_s"]), flush=True)
            os.sched_setaffinity(0, all_cpus)
        print("best GB/s: " + ", ".join("%s/%d: %.2f" % (m, t, best[m, t]) for m in modes for t in counts), flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
