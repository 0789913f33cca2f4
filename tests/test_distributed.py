"""The N>1 path of bench.py on CPU (gloo, world_size 2 and 3): every rank renders
its row-cyclic tiles, rank 0 gathers them and un-interleaves; the result must equal
a single full-frame render.  The per-rank render here is the oracle restricted to the
rank's rows (the device launch is covered by test_gpu_parity's tile test); what this
checks is the partition / gather / reassembly logic and the collective pattern."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, SPP, TILE = 40, 37, 2, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene():
    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl
    r = wl.Renderer("dist", max_nodes=4096)
    info = scenes.build("csg32", r)
    return r, info.params(width=W, height=H, spp=SPP)


def _render_rows(r, p, rows):
    import pyoracle
    prog, nrec, _ = r.program()
    mats, nm = r.materials()
    fr = r.frame_desc(p)
    out = np.zeros((len(rows), W, 4), dtype=np.float32)
    for i, y in enumerate(rows):
        if y < H:
            out[i], _ = pyoracle.pathtrace_rows(prog, nrec, mats, nm, fr, y, 1, nthreads=1)
    return out


def assemble_np(gathered, width, height, tile, n):
    """numpy statement of assemble_kernel (trace_kernels.hip)."""
    from csgrenderer_amd import wololo as wl
    lr = wl.local_rows(height, tile, n)
    frame = np.empty((height, width, 4), dtype=np.float32)
    for y in range(height):
        g = y // tile
        rk = g % n
        lrow = (g // n) * tile + (y - g * tile)
        assert lrow < lr
        frame[y] = gathered[rk, lrow]
    return frame


def _worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WOLOLO_ALLOW_NO_DEVICE="1")
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    from csgrenderer_amd import wololo as wl
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, p = _scene()
    lr = wl.local_rows(H, TILE, world)
    rows = [wl.global_row(l, TILE, rank, world) for l in range(lr)]
    local = torch.from_numpy(_render_rows(r, p, rows))
    gathered = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
    dist.gather(local, gather_list=gathered, dst=0)
    if rank == 0:
        frame = assemble_np(torch.stack(gathered).numpy(), W, H, TILE, world)
        np.save(result_path, frame)
    dist.barrier()
    dist.destroy_process_group()
    r.close()


@pytest.mark.parametrize("world", [2, 3])
def test_row_tiles_gather_assemble(tmp_path, monkeypatch, world):
    monkeypatch.setenv("WOLOLO_ALLOW_NO_DEVICE", "1")
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    frame = np.load(out)
    r, p = _scene()
    full = _render_rows(r, p, list(range(H)))
    assert np.array_equal(frame, full)
    r.close()


@pytest.mark.parametrize("height,tile,n", [(1080, 16, 1), (1080, 16, 8), (2160, 16, 8), (1080, 4, 8), (2160, 4, 8), (1080, 4, 7), (37, 8, 3), (5, 16, 4)])
def test_partition_covers_every_row_once(height, tile, n):
    from csgrenderer_amd import wololo as wl
    lr = wl.local_rows(height, tile, n)
    seen = []
    for rank in range(n):
        for l in range(lr):
            y = wl.global_row(l, tile, rank, n)
            if y < height:
                seen.append(y)
    assert sorted(seen) == list(range(height))
    # load balance: ranks own tile counts that differ by at most one
    tiles = (height + tile - 1) // tile
    counts = [len(range(rank, tiles, n)) for rank in range(n)]
    assert max(counts) - min(counts) <= 1
