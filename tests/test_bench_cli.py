"""bench.py's launcher contract on CPU (no GPU needed): `--gpus N` either runs N
ranks or exits non-zero before touching a device.

  * no launcher and N > 1: bench starts torch.distributed.run with N processes
    itself (checked here by intercepting the child command);
  * a launcher whose WORLD_SIZE differs from --gpus: exit 2;
  * more ranks than visible GPUs without --stack-ranks: exit 2;
  * --single-process under a launcher: exit 2.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=120)


def test_too_few_gpus_exits_2():
    p = _run(["--gpus", "2"])  # this container has no GPU
    assert p.returncode == 2, p.stderr[-2000:]
    assert "needs 2 GPUs" in p.stderr


def test_world_size_mismatch_exits_2():
    p = _run(["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "3 ranks are running" in p.stderr, p.stderr[-2000:]


def test_single_process_under_launcher_exits_2():
    p = _run(["--gpus", "2", "--single-process"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "one process" in p.stderr, p.stderr[-2000:]


def test_single_process_too_few_gpus_exits_2():
    p = _run(["--gpus", "2", "--single-process"])
    assert p.returncode == 2 and "needs 2 GPUs" in p.stderr, p.stderr[-2000:]


@pytest.mark.parametrize("n", [2, 8])
def test_self_launch_starts_n_ranks(n, monkeypatch):
    """The command bench starts without a launcher: torch.distributed.run, N processes
    on one node, 127.0.0.1, this script with the same arguments; its exit status is
    bench's."""
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return Done()

    monkeypatch.setattr(bench, "visible_devices", lambda: n)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", str(n), "--steps", "3"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert f"--nproc-per-node={n}" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", str(n), "--steps", "3"] and cmd[-5].endswith("bench.py")
