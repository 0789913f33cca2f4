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
           "--dist-backend", "gloo", "--verify", "--steps", "4", "--warmup", "1", "--no-cpu-baseline",
           "--width", "480", "--height", "270", "--spp", "8"] + (["--frames-in-flight", str(fif)] if fif else [])
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == nranks
    assert line["verified_vs_full_render"] is True
    assert "overlapped" in line["config"]["parallelism"]
    assert line["config"]["frames_in_flight"] == (fif or 2)
    # every rank's segments are counted: the whole frame's
    assert line["segments_per_frame"] > 480 * 270 * 8
