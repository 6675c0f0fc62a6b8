"""Full-size parity: every packet of a BASELINE-sized batch
decoded on the device through the C ABI and compared with the CPU oracle,
records, error arguments and flow hashes bit for bit (bench.full_parity).

C4 (64 M IMIX packets with Dot1Q/QinQ, IPv6, all outputs) and C1
(test_ethernet.pcap tiled to 10 M packets) run the small-packet kernel at the
sizes the bench reports; the default bench line runs the same check on C3
(the 80-VGPR kernel) and C2 (the 4-chunk-window kernel).
"""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["c4", "c1"])
def test_every_packet(gpu_ctx, name):
    import bench
    res = bench.run_config(name, 64 * 2**20, 1, 0, 0, 1, gpu_ctx, check_sample=0, full_check=True)
    full = res["full_parity"]["result"]
    assert full.startswith("bit-exact (all %d packets" % res["n"]), full
