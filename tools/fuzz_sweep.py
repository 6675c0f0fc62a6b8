#!/usr/bin/env python3
"""A wider fuzz sweep than tests/test_gpu_parity.py::test_fuzz: many seeds,
every test parser, with and without layouts, packed at several alignments, and
on every third seed the layer fields through both forms (layouts + extraction,
and the fused launch; tests/test_fields_gpu.check). Each batch is
compared with the oracle bit for bit (tests/configs.assert_same); the first
mismatch is printed with its seed and the run stops.

    python tools/fuzz_sweep.py [--seeds 20] [--packets 30000]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=20)
    ap.add_argument("--first-seed", type=int, default=5000)
    ap.add_argument("--packets", type=int, default=30000)
    ap.add_argument("--hydrate", type=int, default=0, metavar="K",
                    help="every K-th seed also: Hydrate from the one-launch fields result against Hydrate from "
                         "layouts, struct by struct (tests/hydrate_cases.compare), over the seed's first 4000 packets")
    ap.add_argument("--narrow", type=int, default=0, metavar="K",
                    help="every K-th seed also: gpk_decode_batch_narrow against the oracle's narrow form and the "
                         "16-byte decode, every parser (tests/test_narrow_gpu.check_narrow)")
    ap.add_argument("--layouts", default="", type=lambda x: [y for y in x.split(",") if y],
                    help="placements to cycle through: packed, shuffled, reversed, wave_shuffled, gapped, sparse_mix")
    a = ap.parse_args()
    import torch  # noqa: F401  (libgpk runs on torch's HIP runtime)
    import pktutil
    from configs import CONFIGS, assert_same, device_parser, oracle_parser
    from test_fields_gpu import check as fields_check
    from test_gpu_parity import phase_b_layout
    from gopacket_amd import engine
    ctx = engine.Context()
    t0 = time.time()
    n_batches = 0
    for seed in range(a.first_seed, a.first_seed + a.seeds):
        packets = pktutil.fuzz_packets(seed, a.packets)
        align = (1, 2, 4, 16)[seed % 4]
        layout = a.layouts[seed % len(a.layouts)] if a.layouts else "packed"
        if layout == "packed":
            data, off, cap = pktutil.pack(packets, align=align, pad=(seed * 7) % 24)
        else:  # the parity suite's unordered / gapped / sparse placements
            data, off, cap = phase_b_layout(packets, layout)
        for name in sorted(CONFIGS):
            cfg = CONFIGS[name]
            for layouts in (True, False):
                dev = ctx.decode_host(device_parser(cfg), data, off, cap, layouts=layouts)
                ref = oracle_parser(cfg).decode(data, off, cap, nthreads=8, layouts=layouts)
                assert_same(dev, ref, "seed %d align %d %s %s layouts=%s" % (seed, align, layout, name, layouts))
                n_batches += 1
            if seed % 3 == 0 and layout == "packed":
                fields_check(ctx, name, packets, align=align)
                n_batches += 2
            if a.narrow and seed % a.narrow == 0:
                from test_narrow_gpu import check_narrow
                check_narrow(ctx, cfg, data, off, cap, "seed %d align %d %s %s narrow" % (seed, align, layout, name))
                n_batches += 1
        if a.hydrate and seed % a.hydrate == 0:
            import hydrate_cases as H
            from gopacket_amd import gopacket as G
            sub = packets[:4000] + H.hbh_packets(seed, 500)
            batch = G.PacketBatch.from_packets(sub)
            pa, pb = H.parser(), H.parser()
            pa._ctx = pb._ctx = ctx
            ra, rb = pa.DecodeBatch(batch, layouts=True), pb.DecodeBatch(batch, fields=True)
            H.compare(ra, rb, pa, pb, range(len(sub)))
            n_batches += 1
        print("seed %d (%s, align %d): %d parsers x 2 bit-exact, %.0f s" % (seed, layout, align, len(CONFIGS),
                                                                          time.time() - t0),
              flush=True)
    print("fuzz sweep: %d batches of %d packets, all bit-exact" % (n_batches, a.packets), flush=True)


if __name__ == "__main__":
    main()
