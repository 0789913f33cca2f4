"""GPU: executed-work counters (wo_renderer_count_work) -- the counting variant of
each path kernel traces the same paths as the timed kernel (same segment count,
primary segments = pixels x spp), and its counts stay within the brute-force
bounds of SURVEY.md 8(d) (every primitive tested on every segment)."""
import numpy as np
import pytest

from csgrenderer_amd import scenes
from csgrenderer_amd import wololo as wl

pytestmark = pytest.mark.gpu


def _leaves(r):
    prog, nrec, nprim = r.program()
    sph = sum(1 for i in range(nrec) if prog[i].op == wl.WO_LEAF_SPHERE)
    hs = sum(1 for i in range(nrec) if prog[i].op == wl.WO_LEAF_HALFSPACE)
    bounds = sum(1 for i in range(nrec) if prog[i].op == wl.WO_OP_BOUND)
    return sph, hs, bounds


@pytest.mark.parametrize("scene,path", [("csg32", "jit"), ("csg32", "interpreter"), ("csg32_union", "lanes"),
                                        ("csg256_chain", "jit"), ("rtiow_cover", "lanes")])
@pytest.mark.parametrize("nranks", [1, 3])
def test_work_counters(scene, path, nranks):
    import torch
    r = wl.Renderer("work", max_nodes=4096)
    info = scenes.build(scene, r)
    r.set_tracer(path)
    p = info.params(width=160, height=90, spp=4)
    seg = torch.zeros(1, dtype=torch.int64, device="cuda")
    lr = wl.local_rows(p.height, 4, nranks)
    out = torch.zeros((lr, p.width, 4), dtype=torch.float32, device="cuda")  # rows past the frame stay 0
    rank = nranks - 1
    r.render_rows_device(p, out.data_ptr(), 4, rank, nranks, torch.cuda.current_stream().cuda_stream,
                         seg.data_ptr())
    torch.cuda.synchronize()
    assert r.trace_path() == path
    w = r.count_work(p, 4, rank, nranks)
    segs = int(seg.item())
    assert w["segments"] == segs > 0
    rows = sum(1 for lrow in range(lr) if wl.global_row(lrow, 4, rank, nranks) < p.height)
    assert w["primary_segments"] == rows * p.width * p.spp
    sph, hs, nb = _leaves(r)
    passes = segs + w["recollects"]  # a re-collect tests the primitives again
    assert 0 < w["sphere_tests"] <= passes * sph
    assert w["halfspace_tests"] <= passes * hs
    assert w["bound_tests"] <= passes * nb
    assert w["sweep_steps"] <= w["events"]  # each swept event was stored once (or is the overflow key)
    assert w["sweep_steps"] >= segs - w["primary_segments"]  # every bounce follows a hit: >= 1 swept event
    # counting twice gives the same counts (deterministic paths)
    assert r.count_work(p, 4, rank, nranks) == w
    # and the timed kernel still renders the same image afterwards
    again = torch.zeros_like(out)
    r.render_rows_device(p, again.data_ptr(), 4, rank, nranks, torch.cuda.current_stream().cuda_stream, 0)
    torch.cuda.synchronize()
    assert torch.equal(out, again)
    r.close()
