"""include/gpk.h from C (as cgo uses it): the tiny C11 program in tests/c_abi
is compiled against the public header only and linked with -lgpk; its host
mode checks struct layouts (static asserts), error texts, LayerType names and
parser configuration without a GPU."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CDIR = os.path.join(ROOT, "tests", "c_abi")


def build_c_abi_test():
    subprocess.check_call(["make", "-s", "-C", CDIR])
    return os.path.join(CDIR, "gpk_abi_test")


def test_c_abi_host_mode():
    exe = build_c_abi_test()
    out = subprocess.run([exe, "host", os.path.join(ROOT, "tests", "golden", "c_abi")], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "all checks passed" in out.stdout


def test_c_abi_capture_reader_interface():
    """The capture reader's interface beyond ReadPacketData from C, as a cgo
    binding uses it: EPB options (ngread_test.go:2028-2100) and name records
    (ngread_nrb_test.go:50-79) of the reference's own capture files."""
    exe = build_c_abi_test()
    out = subprocess.run([exe, "capture", os.path.join(ROOT, "tests", "golden", "pcapgo")], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "all checks passed (capture)" in out.stdout
