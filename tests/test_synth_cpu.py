"""Synthetic benchmark batches (host generator) checked by the oracle."""
import numpy as np
import pytest

from gopacket_amd import synth
from oracle import oracle as O


def test_deterministic_per_index():
    d1, o1, c1 = synth.host_batch(synth.C4_IMIX, 1000, 500)
    d2, o2, c2 = synth.host_batch(synth.C4_IMIX, 1000, 500)
    assert np.array_equal(d1, d2)
    assert synth.packet(synth.C4_IMIX, 1003) == bytes(d1[o1[3]:o1[3] + c1[3]])
    assert synth.total_bytes(synth.C4_IMIX, 1000, 500) == int(c1.sum())


@pytest.mark.parametrize("cfg,decoders,expect", [
    (synth.C2_UDP64, ["ETHERNET", "IPV4", "UDP", "PAYLOAD"], 0xBA31),
    (synth.C3_TCP1500, ["ETHERNET", "IPV4", "TCP", "PAYLOAD"], 0xB931),
])
def test_fixed_configs(cfg, decoders, expect):
    d, o, c = synth.host_batch(cfg, 0, 20000)
    r = O.OracleParser(17, decoders).decode(d, o, c, nthreads=4, layouts=False)
    rec = r["records"]
    assert np.all(rec["layers"] == expect)            # Eth, IPv4, UDP|TCP, Payload
    st = rec["status"]
    assert np.all(st & 0x7F == 0)
    bad_ip = np.sum(~st & (1 << 21) != 0)
    bad_l4 = np.sum(~st & (1 << 23) != 0)
    assert 0 < bad_ip + bad_l4 < 60                    # ~1/1024 corrupted checksums


def test_imix_mix():
    d, o, c = synth.host_batch(synth.C4_IMIX, 0, 24000)
    vals, cnt = np.unique(c, return_counts=True)
    assert list(vals) == [64, 594, 1518]
    assert abs(cnt[0] / len(c) - 7 / 12) < 0.02 and abs(cnt[2] / len(c) - 1 / 12) < 0.02
    r = O.OracleParser(17, ["ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP", "PAYLOAD"]).decode(
        d, o, c, nthreads=4, layouts=False)
    st = r["records"]["status"]
    assert np.all(st & 0x7F == 0)
    v6 = np.sum((st >> 27) & 1)
    assert 0.1 < v6 / len(c) < 0.2  # 20% IPv6 where IPv6 + UDP fit the frame
