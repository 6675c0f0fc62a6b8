"""C3 with its batch and its outputs in ONE allocation (diagnostic, DESIGN §5
Variance): K fresh arenas in one process, each [batch bytes | index | records |
err | flows] at fixed relative offsets, against K layouts of separate
allocations (the bench's: batch, then outputs). Each timed like
tools/c3_mode.py (2 warm, median of 4 single launches). Does a fixed relative
placement of outputs and inputs fix the mode?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from gopacket_amd import _lib, engine, synth  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ctx = engine.Context(0)
cfg = bench.CONFIGS["c3"]
parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
n = 64 * 2**20
stream = torch.cuda.current_stream()
S = _lib.synth_lib()
total = synth.total_bytes(3, 0, n) + 256


def timeit(data, off, cap, rec, err, fl):
    ts = []
    for j in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ctx.decode_device(parser, data, off, cap, rec, err, fl, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        if j >= 2:
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def align(x, a=1 << 21):
    return (x + a - 1) // a * a


for mode in ("separate", "arena"):
    for k in range(K):
        if mode == "separate":
            data, off, cap = synth.device_batch(3, 0, n, stream=stream)
            rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
            err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
            fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
            t = timeit(data, off, cap, rec, err, fl)
            del data, off, cap, rec, err, fl
        else:
            o_off = align(total)
            o_cap = align(o_off + 8 * n)
            o_rec = align(o_cap + 4 * n)
            o_err = align(o_rec + 16 * n)
            o_fl = align(o_err + 8 * n)
            arena = torch.empty(align(o_fl + 24 * n), dtype=torch.uint8, device="cuda")
            data = arena[:total]
            off = arena[o_off:o_off + 8 * n].view(torch.int64)
            cap = arena[o_cap:o_cap + 4 * n].view(torch.int32)
            assert S.gpk_synth_device(3, 0, n, data.data_ptr(), off.data_ptr(), cap.data_ptr(), stream.cuda_stream) == 0
            rec = arena[o_rec:o_rec + 16 * n]
            err = arena[o_err:o_err + 8 * n].view(torch.int32)
            err.zero_()
            fl = arena[o_fl:o_fl + 24 * n].view(torch.int64)
            t = timeit(data, off, cap, rec, err, fl)
            del arena, data, off, cap, rec, err, fl
        torch.cuda.empty_cache()
        print("%s %d: %.3f ms" % (mode, k, t), flush=True)
