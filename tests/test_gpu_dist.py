"""GPU: the N>1 bench path rehearsed on one GPU.

bench.py runs frames pipelined -- frame k+1 renders on a second stream into the
other of two buffers while frame k is gathered, ordered by events -- with either
backend.  Here torchrun starts N ranks on this one GPU with the gloo backend (RCCL
refuses two ranks on one device), so the two-buffer / two-stream / event code the
driver's 8-GPU RCCL run executes runs here, and rank 0 checks the assembled frame
against one full-frame render bit for bit (--verify).  The test process itself
only starts the child processes."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("nranks,fif", [(2, None), (8, None), (2, 1)])
def test_pipelined_rehearsal_verifies(nranks, fif):
    """N ranks, frames pipelined with the gather; by default two frames in flight on
    two render streams (fif None), and with one render stream (fif 1)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(nranks),
           "--dist-backend", "gloo", "--stack-ranks", "--verify", "--steps", "4", "--warmup", "1", "--no-cpu-baseline",
           "--width", "480", "--height", "270", "--spp", "8"] + (["--frames-in-flight", str(fif)] if fif else [])
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == nranks
    assert line["config"]["ranks"] == nranks and line["config"]["devices"] == 1
    assert "stacked" in line["config"]["parallelism"]
    assert line["verified_vs_full_render"] is True
    assert "overlapped" in line["config"]["parallelism"]
    assert line["config"]["frames_in_flight"] == (fif or 2)
    # every rank's segments are counted: the whole frame's
    assert line["segments_per_frame"] > 480 * 270 * 8


def _bench_line(cmd, timeout=150):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


SMALL = ["--steps", "4", "--warmup", "1", "--no-cpu-baseline", "--width", "480", "--height", "270", "--spp", "8"]


@pytest.mark.parametrize("nranks", [2, 3])
def test_single_process_mode_verifies(nranks):
    """bench.py --single-process: one process, N ranks through wo_renderer_set_devices
    (stacked on this GPU), every step a wo_renderer_render_frame_device; the last frame
    equals a one-rank render bit for bit and the line names N ranks."""
    line = _bench_line([sys.executable, "bench.py", "--gpus", str(nranks), "--single-process", "--stack-ranks",
                        "--verify"] + SMALL)
    assert line["n_gpus"] == nranks and line["config"]["ranks"] == nranks
    assert line["config"]["launcher"] == "single-process"
    assert line["verified_vs_full_render"] is True
    assert line["segments_per_frame"] > 480 * 270 * 8


def test_self_launch_without_a_launcher():
    """`bench.py --gpus 2` with no torchrun: bench starts torch.distributed.run itself
    (here with stacked gloo ranks), and the line reports the 2 ranks that ran."""
    line = _bench_line([sys.executable, "bench.py", "--gpus", "2", "--stack-ranks", "--dist-backend", "gloo",
                        "--verify"] + SMALL)
    assert line["n_gpus"] == 2 and line["config"]["launcher"] == "torchrun"
    assert line["verified_vs_full_render"] is True


def test_rank_mismatch_fails_loudly():
    """--gpus 2 on one GPU without --stack-ranks: exit status 2 before any rank starts."""
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2"] + SMALL, cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 2 and "needs 2 GPUs" in p.stderr, p.stderr[-2000:]
