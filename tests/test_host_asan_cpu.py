"""The host parsers of untrusted input under AddressSanitizer + UBSan: the
pcap/pcapng capture reader and the AF_PACKET ring walk, compiled from the
product sources into tests/asan/build/fuzz_host and driven over mutated
capture files (the reference's own pcapgo fixtures and the pcap test files as
seeds) and randomly corrupted V1/V2/V3 rings (tests/asan/fuzz_host.cpp).
A sanitizer report, a broken API contract or a hang fails the test."""
import glob
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ASAN = os.path.join(HERE, "asan")


def _seeds():
    g = os.path.join(HERE, "golden")
    return sorted(glob.glob(os.path.join(g, "pcapgo", "le", "*.pcapng")) +
                  glob.glob(os.path.join(g, "pcapgo", "be", "*.pcapng")) +
                  [os.path.join(g, "pcapgo", "epb.pcapng"), os.path.join(g, "test_ethernet.pcap"),
                   os.path.join(g, "test_dns.pcap")])


@pytest.fixture(scope="module")
def fuzz_host():
    if not shutil.which("g++") or not os.path.exists("/opt/rocm/include/hip/hip_runtime.h"):
        pytest.skip("needs g++ and the HIP headers")
    r = subprocess.run(["make", "-C", ASAN], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(ASAN, "build", "fuzz_host")


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_capture_reader_and_ring_walk_under_asan(fuzz_host, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:handle_abort=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([fuzz_host, str(seed), "20000"] + _seeds(), capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0 and "ERROR" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert "fuzz_host ok" in r.stdout
