"""bench.py's launch decision for `--gpus N`: N > 1
without a launcher starts torch.distributed.run as a child; under a launcher
the world size must equal N. Also the relay of the child's output."""
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_one_gpu_runs_in_process():
    b = _bench()
    assert b.launch_plan(1, {}, ["--gpus", "1"]) == ("inproc", None)


def test_n_gpus_without_launcher_spawns_torchrun_child():
    b = _bench()
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "2"]
    mode, cmd = b.launch_plan(8, {}, argv, port=29555)
    assert mode == "spawn"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    j = [k for k, x in enumerate(cmd) if x.endswith("bench.py")][0]
    assert cmd[j + 1:] == argv  # the same arguments reach every rank


def test_under_launcher_world_must_match():
    b = _bench()
    assert b.launch_plan(2, {"WORLD_SIZE": "2"}, []) == ("inproc", None)
    with pytest.raises(SystemExit):
        b.launch_plan(8, {"WORLD_SIZE": "1"}, [])
    with pytest.raises(SystemExit):
        b.launch_plan(1, {"WORLD_SIZE": "2"}, [])
    with pytest.raises(SystemExit):
        b.launch_plan(0, {}, [])


def test_relay_passes_output_and_exit_status(capsys):
    b = _bench()
    ok = [sys.executable, "-c", "print('rank log'); print('{\"value\": 1}')"]
    assert b.spawn_ranks(ok) == 0
    out = capsys.readouterr().out
    assert "rank log" in out and '{"value": 1}' in out
    # a child that fails passes its status through
    assert b.spawn_ranks([sys.executable, "-c", "import sys; sys.exit(3)"]) == 3
    # a child that exits 0 without its JSON line is a failure
    assert b.spawn_ranks([sys.executable, "-c", "print('no line')"]) == 1


def test_bench_world_mismatch_fails_before_the_gpu():
    """A rank whose launcher's world size differs from --gpus exits non-zero
    (no GPU needed: it stops before importing torch)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--configs", "c2", "--packets", "4096"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr


def test_terminating_the_parent_ends_the_ranks(tmp_path):
    """A driver's timeout sends SIGTERM to `bench.py --gpus N`: the torchrun
    child (and with it the ranks) is terminated and reaped, not orphaned."""
    import signal
    import subprocess
    import time
    script = tmp_path / "parent.py"
    script.write_text(
        "import importlib.util, sys\n"
        "spec = importlib.util.spec_from_file_location('b', %r)\n"
        "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
        "sys.exit(b.spawn_ranks([sys.executable, '-u', '-c', "
        "'import os, time; print(os.getpid(), flush=True); time.sleep(120)']))\n" % os.path.join(ROOT, "bench.py"))
    p = subprocess.Popen([sys.executable, "-u", str(script)], stdout=subprocess.PIPE, text=True)
    child = int(p.stdout.readline())
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=60) == 128 + signal.SIGTERM
    deadline = time.time() + 10
    while True:
        try:
            os.kill(child, 0)
        except ProcessLookupError:
            break
        assert time.time() < deadline, "the child outlived its parent"
        time.sleep(0.1)
