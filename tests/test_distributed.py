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


def assemble_np(gathered, width, height, tile, n, band=(0, 0)):
    """numpy statement of assemble_kernel (trace_kernels.hip): frame row y is row
    lb * tile + y mod tile of the rank whose local band lb is frame band y div tile."""
    from csgrenderer_amd import wololo as wl
    lr = wl.local_rows(height, tile, n, band)
    owner = {}
    for rk in range(n):
        for lb in range(lr // tile):
            owner[wl.band_global(lb, rk, n, band)] = (rk, lb)
    frame = np.empty((height, width, 4), dtype=np.float32)
    for y in range(height):
        g = y // tile
        rk, lb = owner[g]
        lrow = lb * tile + (y - g * tile)
        assert lrow < lr
        frame[y] = gathered[rk, lrow]
    return frame


def _worker(rank, world, port, result_path, band):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WOLOLO_ALLOW_NO_DEVICE="1")
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    from csgrenderer_amd import wololo as wl
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, p = _scene()
    lr = wl.local_rows(H, TILE, world, band)
    rows = [wl.global_row(l, TILE, rank, world, band) for l in range(lr)]
    local = torch.from_numpy(_render_rows(r, p, rows))
    gathered = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
    dist.gather(local, gather_list=gathered, dst=0)
    if rank == 0:
        frame = assemble_np(torch.stack(gathered).numpy(), W, H, TILE, world, band)
        np.save(result_path, frame)
    dist.barrier()
    dist.destroy_process_group()
    r.close()


@pytest.mark.parametrize("world,band", [(2, (0, 0)), (3, (0, 0)), (3, (2, 1))])
def test_row_tiles_gather_assemble(tmp_path, monkeypatch, world, band):
    """(band: rank 0 sitting out `skip` of every `cycle` rounds of bands, bench.py's
    weighting of the root's share)"""
    monkeypatch.setenv("WOLOLO_ALLOW_NO_DEVICE", "1")
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), out, band), nprocs=world, join=True,
                       start_method="spawn")
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


@pytest.mark.parametrize("height,tile,n,band", [(1080, 4, 8, (8, 1)), (1080, 4, 4, (16, 1)), (1080, 4, 2, (32, 1)),
                                                (2160, 4, 8, (8, 2)), (37, 8, 3, (2, 1)), (5, 16, 4, (8, 1)),
                                                (1080, 4, 8, (5, 4))])
def test_weighted_bands_cover_every_row_once(height, tile, n, band):
    """Weighted bands (wo_band_global): every frame row once, rank 0 owning
    (cycle - skip) / cycle of another rank's bands over whole cycles."""
    from csgrenderer_amd import wololo as wl
    lr = wl.local_rows(height, tile, n, band)
    seen = []
    counts = []
    for rank in range(n):
        rows = [wl.global_row(l, tile, rank, n, band) for l in range(lr)]
        owned = [y for y in rows if y < height]
        assert owned == sorted(owned) and len(owned) <= lr
        assert wl.rank_bands(height, tile, rank, n, band) == (len(owned) + tile - 1) // tile
        counts.append(wl.rank_bands(height, tile, rank, n, band))
        seen += owned
    assert sorted(seen) == list(range(height))
    tiles = (height + tile - 1) // tile
    cycle, skip = band
    full_cycles = tiles // (cycle * n - skip)
    if full_cycles:
        assert counts[0] >= full_cycles * (cycle - skip) and min(counts[1:]) >= full_cycles * cycle


def test_band_mapping_matches_the_header(tmp_path):
    """wololo.py's band mirrors equal wo_scene.h's inline C (compiled here with gcc)."""
    import subprocess
    from csgrenderer_amd import wololo as wl
    src = tmp_path / "b.c"
    src.write_text('''#include <stdio.h>
#include "wololo/wo_scene.h"
int main(void) {
    const unsigned cases[][4] = {{1080, 4, 8, 8}, {1080, 4, 4, 16}, {37, 8, 3, 2}, {2160, 4, 8, 8}, {1080, 4, 7, 3}};
    for (int i = 0; i < 5; ++i)
        for (unsigned skip = 0; skip < 3; ++skip) {
            unsigned H = cases[i][0], T = cases[i][1], n = cases[i][2], cyc = cases[i][3];
            printf("%u", wo_rank_local_rows_ex(H, T, n, cyc, skip));
            for (unsigned r = 0; r < n; ++r) {
                printf(" %u", wo_rank_tile_count_ex(H, T, r, n, cyc, skip));
                for (unsigned lb = 0; lb < 40; ++lb) printf(" %u", wo_band_global(lb, r, n, cyc, skip));
            }
            printf("\\n");
        }
    return 0;
}
''')
    exe = tmp_path / "b"
    subprocess.run(["gcc", "-std=gnu11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    lines = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    k = 0
    for H_, T_, n_, cyc in [(1080, 4, 8, 8), (1080, 4, 4, 16), (37, 8, 3, 2), (2160, 4, 8, 8), (1080, 4, 7, 3)]:
        for skip in range(3):
            want = [wl.local_rows(H_, T_, n_, (cyc, skip))]
            for r in range(n_):
                want.append(wl.rank_bands(H_, T_, r, n_, (cyc, skip)))
                want += [wl.band_global(lb, r, n_, (cyc, skip)) for lb in range(40)]
            assert [int(x) for x in lines[k].split()] == want, (H_, T_, n_, cyc, skip)
            k += 1
