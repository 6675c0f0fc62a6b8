"""Two parsers with different next-layer tables used alternately on two HIP
streams with no synchronisation between calls: each launch must see its own
parser's tables (gopacket gives every parser its own state, doc.go:211-228;
port overrides as RegisterTCPPortLayerType / RegisterUDPPortLayerType make
them, ports.go:99-104). Checked bit for bit against the oracle."""
import numpy as np
import pytest

import pktutil
from configs import CONFIGS, device_parser, oracle_parser

pytestmark = pytest.mark.gpu


def test_alternating_parsers_on_two_streams(gpu_ctx):
    import torch
    from gopacket_amd import _lib
    g = pktutil.golden()
    base = [bytes.fromhex(v["hex"]) for k, v in sorted(g.items()) if "hex" in v]
    base += pktutil.read_pcap(pktutil.GOLDEN + "/test_ethernet.pcap")[1]
    base += pktutil.read_pcap(pktutil.GOLDEN + "/test_dns.pcap")[1]
    base += pktutil.fuzz_packets(77, 4000)
    reps = (8 << 20) // len(base) + 1
    n1 = len(base)
    data1, off1, cap1 = pktutil.pack(base)
    # the batch: the unique set tiled `reps` times (oracle decodes the unique set once)
    span = int(off1[-1]) + int(cap1[-1])
    n = n1 * reps
    data = np.zeros(span * reps + 64, np.uint8)
    for r in range(reps):
        data[r * span:(r + 1) * span] = data1[:span]
    off = (np.tile(off1.astype(np.uint64), reps) + np.repeat(np.arange(reps, dtype=np.uint64) * span, n1))
    cap = np.tile(cap1, reps)
    names = ("overrides", "eth_ip4_udp_payload")
    refs = {k: oracle_parser(CONFIGS[k]).decode(data1, off1, cap1, nthreads=8) for k in names}
    assert not np.array_equal(refs[names[0]]["records"], refs[names[1]]["records"])
    parsers = {k: device_parser(CONFIGS[k]) for k in names}
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.astype(np.int64)).cuda()
    c = torch.from_numpy(cap.astype(np.int32)).cuda()
    streams = {k: torch.cuda.Stream() for k in names}
    outs = []
    torch.cuda.synchronize()
    for it in range(3):
        for k in names:
            rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
            err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
            fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
            with torch.cuda.stream(streams[k]):
                gpu_ctx.decode_device(parsers[k], d, o, c, rec, err, fl, stream=streams[k])
            outs.append((k, rec, err, fl))
    torch.cuda.synchronize()
    for k, rec, err, fl in outs:
        ref = refs[k]
        got = rec.cpu().numpy().view(_lib.RECORD_DTYPE)
        assert np.array_equal(got, np.tile(ref["records"], reps)), k
        rf = ref["flows"].reshape(3, n1)
        assert np.array_equal(fl.cpu().numpy().view(np.uint64).reshape(3, n), np.tile(rf, (1, reps))), k
        e = (got["status"] & 0x7F) != 0
        assert np.array_equal(err.cpu().numpy().view(np.uint32).reshape(n, 2)[e],
                              np.tile(ref["err_args"].reshape(n1, 2), (reps, 1))[e]), k
