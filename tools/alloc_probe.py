#!/usr/bin/env python3
"""Does where the batch and the outputs live change the decode's rate?

Same kernel, same packets; the packed batch in a torch allocation or in
physically contiguous device memory (hipDeviceMallocContiguous), the outputs
(records, error arguments, flows) in a torch allocation, uncached device
memory (hipDeviceMallocUncached: stores go past the L2) or fine-grained
device memory. Interleaved rounds in one process, HIP-event kernel time,
every combination's outputs compared with the first's; the batch is
allocated twice per kind to show the spread between allocations.

    python tools/alloc_probe.py --configs c3,c4,c2 --rounds 4 --steps 5
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FLAGS = {"hip": 0, "contig": 4, "uncached": 3, "fine": 1}


class Raw:
    """A device buffer from gpk_probe_malloc, with the two methods the engine reads."""

    def __init__(self, S, nbytes, flags, elsize=1):
        self.S, self.p, self.n, self.el = S, ctypes.c_void_p(), nbytes // elsize, elsize
        if S.gpk_probe_malloc(ctypes.byref(self.p), nbytes, flags) != 0:
            raise MemoryError("gpk_probe_malloc(%d, %d)" % (nbytes, flags))

    def data_ptr(self):
        return self.p.value

    def numel(self):
        return self.n

    def free(self):
        if self.p.value:
            self.S.gpk_probe_free(self.p)
            self.p = ctypes.c_void_p()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c4,c2")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--instances", default="torch+contig",
                    help="comma-separated batch allocation sets, each kinds joined by + in allocation order "
                         "(torch, hip = hipMalloc-equivalent flags 0, contig); one set live at a time")
    ap.add_argument("--outs", default="torch,uncached,fine")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from gopacket_amd import _lib, engine, synth
    S = _lib.synth_lib()
    ctx = engine.Context(0)
    stream = torch.cuda.current_stream()
    for name in a.configs.split(","):
        cfg = bench.CONFIGS[name]
        if "synth" not in cfg:
            continue
        n = 64 * 2**20
        total = synth.total_bytes(cfg["synth"], 0, n) + 256
        parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
        zero = torch.zeros(24 * n, dtype=torch.uint8, device="cuda")
        outs = {}
        out_kinds = a.outs.split(",")
        for kind in out_kinds:
            if kind == "torch":
                outs[kind] = (torch.empty(n * 16, dtype=torch.uint8, device="cuda"),
                              torch.zeros(2 * n, dtype=torch.int32, device="cuda"),
                              torch.empty(3 * n, dtype=torch.int64, device="cuda"))
            else:
                outs[kind] = (Raw(S, n * 16, FLAGS[kind]), Raw(S, 8 * n, FLAGS[kind], 4), Raw(S, 24 * n, FLAGS[kind], 8))
                for x, nb in zip(outs[kind], (n * 16, 8 * n, 24 * n)):  # error arguments are written only on errors
                    assert S.gpk_probe_d2d(x.data_ptr(), zero.data_ptr(), nb) == 0
        del zero
        for inst, spec in enumerate(a.instances.split(",")):
            datas = {}
            for kind in spec.split("+"):
                if kind == "torch":
                    d = torch.empty(total, dtype=torch.uint8, device="cuda")
                    o = torch.empty(n, dtype=torch.int64, device="cuda")
                    c = torch.empty(n, dtype=torch.int32, device="cuda")
                else:
                    try:
                        d = Raw(S, total, FLAGS[kind])
                    except MemoryError as e:
                        print("%-3s alloc %d  data %-6s: %s" % (name, inst, kind, e), flush=True)
                        continue
                    o, c = Raw(S, 8 * n, FLAGS[kind], 8), Raw(S, 4 * n, FLAGS[kind], 4)
                assert S.gpk_synth_device(cfg["synth"], 0, n, d.data_ptr(), o.data_ptr(), c.data_ptr(),
                                          stream.cuda_stream) == 0
                datas[kind] = (d, o, c)
            torch.cuda.synchronize()
            algo = (total - 256) + 12 * n
            combos = [(dk, ok) for dk in datas for ok in out_kinds]
            times = {k: [] for k in combos}
            for rnd in range(a.rounds + 1):
                for k in combos:
                    d, o, c = datas[k[0]]
                    rec, err, fl = outs[k[1]]
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(a.steps):
                        ctx.decode_device(parser, d, o, c, rec, err, fl, stream=stream)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    if rnd:
                        times[k].append(e0.elapsed_time(e1) / a.steps)
            # outputs: every combination's against the first's
            ref = None
            for k in combos:
                d, o, c = datas[k[0]]
                rec, err, fl = outs[k[1]]
                r = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
                e = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
                f = torch.empty(3 * n, dtype=torch.int64, device="cuda")
                ctx.decode_device(parser, d, o, c, rec, err, fl, stream=stream)
                torch.cuda.synchronize()
                for src, dst, nb in ((rec, r, n * 16), (err, e, 8 * n), (fl, f, 24 * n)):
                    assert S.gpk_probe_d2d(dst.data_ptr(), src.data_ptr(), nb) == 0
                torch.cuda.synchronize()
                out = (r, e, f)
                if ref is None:
                    ref = out
                    same = True
                else:
                    same = all(torch.equal(x, y) for x, y in zip(ref, out))
                t = np.array(times[k])
                print("%-3s alloc %d  data %-6s out %-8s median %8.3f ms  min %8.3f  %6.1f%% of 8 TB/s  outputs %s"
                      % (name, inst, k[0], k[1], np.median(t), t.min(), algo / (np.median(t) * 1e-3) / 8e12 * 100,
                         "equal" if same else "DIFFER"), flush=True)
            del ref, out, r, e, f, d, o, c, rec, err, fl
            for kind in datas:
                if kind != "torch":
                    for x in datas[kind]:
                        x.free()
            del datas
            torch.cuda.empty_cache()
        for kind in out_kinds:
            if kind != "torch":
                for x in outs[kind]:
                    x.free()
        del outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
