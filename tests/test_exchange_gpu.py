"""gpk_pack_batch (the send side of the flow exchange) against numpy on
fuzzed and synthetic packets; exchange_packets over RCCL with one rank on the
GPU (all-to-alls of device tensors through the nccl backend)."""
import os
import socket

import numpy as np
import pytest

import pktutil
from gopacket_amd import flows, shard, synth

pytestmark = pytest.mark.gpu


def test_pack_batch_matches_numpy(gpu_ctx):
    import torch
    pk = pktutil.fuzz_packets(77, 5000) + [b""] * 3
    data, off, cap = pktutil.pack(pk, align=7, pad=5)
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.astype(np.int64)).cuda()
    c = torch.from_numpy(cap.astype(np.int32)).cuda()
    rng = np.random.default_rng(2)
    order = rng.permutation(len(pk))[:4000].astype(np.int32)
    od, oo, oc = flows.pack_batch(d, o, c, torch.from_numpy(order).cuda())
    torch.cuda.synchronize()
    od, oo, oc = od.cpu().numpy(), oo.cpu().numpy(), oc.cpu().numpy()
    assert np.array_equal(oc, cap[order].astype(np.int32))
    assert np.array_equal(oo, np.concatenate([[0], np.cumsum(cap[order], dtype=np.int64)[:-1]]))
    for j in range(0, len(order), 13):
        assert bytes(od[oo[j]:oo[j] + oc[j]]) == pk[order[j]]


def test_exchange_over_rccl_single_rank(gpu_ctx):
    import torch
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        d, o, c = synth.device_batch(6, 0, 20000)
        dest = torch.zeros(20000, dtype=torch.int64, device="cuda")
        dest[::5] = -1  # dropped
        rd, ro, rc, src, idx = shard.exchange_packets(d, o, c, dest, 1)
        torch.cuda.synchronize()
        keep = np.nonzero(dest.cpu().numpy() >= 0)[0]
        assert np.array_equal(idx.cpu().numpy(), keep) and np.all(src.cpu().numpy() == 0)
        hd, ho, hc = synth.host_batch(6, 0, 20000)
        rdn, ron, rcn = rd.cpu().numpy(), ro.cpu().numpy(), rc.cpu().numpy()
        for j in range(0, len(keep), 17):
            i = keep[j]
            assert bytes(rdn[ron[j]:ron[j] + rcn[j]]) == bytes(hd[ho[i]:ho[i] + hc[i]])
    finally:
        dist.destroy_process_group()
