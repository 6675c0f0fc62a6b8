"""The C-language caller decodes the golden packets (reference vectors, the
reference's capture files, fuzzed packets) through gpk_decode_batch_host and
compares records, error arguments, flow hashes and Go error texts with the
committed oracle expectations (tools/make_c_abi_golden.py)."""
import os
import subprocess

import pytest

from test_c_abi_cpu import ROOT, build_c_abi_test

pytestmark = pytest.mark.gpu


def test_c_abi_decode_mode():
    exe = os.path.join(ROOT, "tests", "c_abi", "gpk_abi_test")
    if not os.path.exists(exe):  # built by __graft_entry__.build(); the box has gcc too
        exe = build_c_abi_test()
    out = subprocess.run([exe, "decode", os.path.join(ROOT, "tests", "golden", "c_abi")], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "all checks passed (decode)" in out.stdout
    assert "statsassembly: 639 packets" in out.stdout
    assert "fields records checked" in out.stdout


def test_c_abi_replay_with_fields(tmp_path):
    """The C caller drives gpk_replay_file with gpk_replay_opts.fields_cb over a
    synthetic C4 capture and the reference's own capture files: results in
    packet order, every batch's fields before its records, the packet count
    equal to the capture reader's, and for every packet decoded without error
    the fields' present bits equal to the decoders its decoded list names."""
    from gopacket_amd import _lib
    exe = os.path.join(ROOT, "tests", "c_abi", "gpk_abi_test")
    if not os.path.exists(exe):
        exe = build_c_abi_test()
    synth = str(tmp_path / "c4.pcapng")
    assert _lib.synth_lib().gpk_synth_write_pcapng(synth.encode(), 4, 5, 20000, 4) > 0
    g = os.path.join(ROOT, "tests", "golden")
    files = [synth] + [os.path.join(g, "pcapgo", "le", "test%03d.pcapng" % k) for k in (1, 5, 10)] + \
        [os.path.join(g, "pcapgo", "epb.pcapng"), os.path.join(g, "test_ethernet.pcap")]
    out = subprocess.run([exe, "replay"] + files, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "all checks passed (replay)" in out.stdout
    import re
    m = re.search(r"replay c4\.pcapng: (\d+) packets, (\d+) checked", out.stdout)
    assert m and int(m.group(1)) == 20000 and int(m.group(2)) > 15000, out.stdout


@pytest.mark.parametrize("threads,copies,reps", [(4, 400, 3), (8, 150, 2)])
def test_c_abi_threads_contexts(threads, copies, reps):
    """The Go-shaped multi-GPU caller: one process, four
    OS threads, a gpk_ctx + parser per thread on device t % ndev (four
    contexts on the test box's one GPU), each decoding its byte-balanced slice
    of one batch concurrently: host buffers, device buffers on a stream of its
    own, and a context shared by all four. The slices put back together equal
    one context's decode bit for bit, that decode equals the committed oracle
    expectations for every packet, and after every gpk_* call the thread's
    current HIP device is the one it set before the call. Also 8 threads."""
    exe = os.path.join(ROOT, "tests", "c_abi", "gpk_threads_test")
    if not os.path.exists(exe):
        build_c_abi_test()
    out = subprocess.run([exe, os.path.join(ROOT, "tests", "golden", "c_abi"), str(threads), str(copies), str(reps)],
                         capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "all checks passed (threads)" in out.stdout
    assert ", 0 differ from the oracle" in out.stdout, out.stdout
    assert "per-thread host bit-exact, device bit-exact, shared bit-exact" in out.stdout, out.stdout


@pytest.mark.parametrize("threads", [3, 8])
def test_c_abi_threads_replay_ranges(tmp_path, threads):
    """C5's Go shape on N GPUs in one process: a thread and a context per byte
    range of one pcapng (gpk_replay_file_range), all replaying at once (the
    replay pipeline's reader threads, staging, device walk and launches of
    several contexts side by side); the ranges' results concatenated equal one
    context's whole-file replay bit for bit (records, error arguments, flows,
    capture info, capture lengths), every range clean, every thread's device
    kept."""
    from gopacket_amd import _lib
    exe = os.path.join(ROOT, "tests", "c_abi", "gpk_threads_test")
    if not os.path.exists(exe):
        build_c_abi_test()
    path = str(tmp_path / "c4.pcapng")
    assert _lib.synth_lib().gpk_synth_write_pcapng(path.encode(), 4, 77, 200000, 4) > 0
    out = subprocess.run([exe, "replay", path, str(threads)], capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "all checks passed (threads replay)" in out.stdout
    assert "= 200000 of 200000, bit-exact" in out.stdout, out.stdout
    assert "stop: in a callback after 2 of 200 batches" in out.stdout, out.stdout  # gpk_stop, C caller
