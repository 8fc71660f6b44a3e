"""CPU: bench.py --gpus N starts its own N rank processes when no launcher set WORLD_SIZE (bench.py launch_ranks):
each gets torchrun's environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), rank 0's
stdout carries the one JSON line, and a failing rank makes the launcher stop the others and return non-zero.
The rank program here is tests/launch_probe.py (gloo, no model); the GPU test
(tests/test_gpu_bench_launcher.py) runs bench.py itself."""
import json
import os
import subprocess
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tests", "launch_probe.py")


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def test_launcher_starts_world_of_ranks(capfd):
    b = _bench()
    a = types.SimpleNamespace(gpus=3, same_device=True)
    rc = b.launch_ranks(a, script=PROBE, argv=[])
    out = capfd.readouterr().out.strip().splitlines()
    assert rc == 0
    line = json.loads(out[-1])
    assert line == {"world": 3, "sum_of_ranks": 3.0, "local_rank": 0, "master_addr": "127.0.0.1"}
    assert sum(l.startswith("{") for l in out) == 1, "only rank 0 prints the JSON line"


def test_launcher_propagates_a_failing_rank(capfd):
    b = _bench()
    a = types.SimpleNamespace(gpus=2, same_device=True)
    rc = b.launch_ranks(a, script=PROBE, argv=["--fail-rank", "1"])
    capfd.readouterr()
    assert rc == 3


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "initialised world size is 1" in r.stderr


def test_launcher_starts_world_of_eight_ranks(capfd):
    """The 8-GPU node's world (the driver's SCALE run), rehearsed with 8 gloo rank processes on the CPU."""
    b = _bench()
    a = types.SimpleNamespace(gpus=8, same_device=True)
    rc = b.launch_ranks(a, script=PROBE, argv=[])
    out = capfd.readouterr().out.strip().splitlines()
    assert rc == 0
    line = json.loads(out[-1])
    assert line == {"world": 8, "sum_of_ranks": 28.0, "local_rank": 0, "master_addr": "127.0.0.1"}
    assert sum(l.startswith("{") for l in out) == 1


def test_launcher_stops_seven_ranks_when_one_fails(capfd):
    b = _bench()
    a = types.SimpleNamespace(gpus=8, same_device=True)
    rc = b.launch_ranks(a, script=PROBE, argv=["--fail-rank", "5"])
    capfd.readouterr()
    assert rc == 3
