"""Scene-specialised kernels (csrc/scene_jit.c): the generated HIP source compiles
for gfx950 with hiprtc (no GPU needed) and mirrors the compiled program (CPU)."""
import re

import numpy as np
import pytest

from csgrenderer_amd import scenes
from csgrenderer_amd import wololo as wl


def test_csg32_source_compiles_for_gfx950(hostonly):
    r = wl.Renderer("jit", max_nodes=4096)
    scenes.build("csg32", r)
    prog, nrec, nprim = r.program()
    src = r.jit_source()
    assert src is not None
    # one intersection call per leaf (a slab's two opposite faces: one pair call) in
    # each of the two collect passes (first pass, re-collect), one cull flag per
    # BOUND, ordinal table of every primitive
    nleaf = sum(1 for i in range(nrec) if prog[i].op in (wl.WO_LEAF_SPHERE, wl.WO_LEAF_HALFSPACE))
    nsingle = len(re.findall(r"wodev::(sphere|halfspace|halfspace_axis)_interval\(", src))
    npair = len(re.findall(r"wodev::axis_pair_meet\(", src))
    assert npair >= 2 * 6  # the slab and the cube: three face pairs each, in both passes
    assert nsingle + 2 * npair == 2 * nleaf
    # the slab and the cube are axis-aligned: tagged by the compiler, emitted on the fast path
    naxis = sum(1 for i in range(nrec) if prog[i].op == wl.WO_LEAF_HALFSPACE and prog[i].u1 != 0)
    assert naxis >= 12
    assert len(re.findall(r"wodev::halfspace_axis_interval\(", src)) + 2 * npair == 2 * naxis
    # wave-level tests only for BOUND subtrees of >= 6 leaves (scene_jit.c, WOLOLO_JIT_BOUND_MIN_LEAVES)
    # and not around a lone primitive (WOLOLO_JIT_BOUND_SINGLE=0: its member skip is the cheaper test)
    def lone(i):
        return prog[i + 1].op == wl.WO_OP_PRIM and i + 2 + prog[i + 1].u0 == prog[i].u0

    nb = sum(1 for i in range(nrec) if prog[i].op == wl.WO_OP_BOUND and prog[i].u1 >= 6 and not lone(i))
    assert 0 < nb < sum(1 for i in range(nrec) if prog[i].op == wl.WO_OP_BOUND)
    assert len(re.findall(r"if \(__ballot\(wodev::bound_may_hit\(", src)) == nb
    m = re.search(r"kOrdPc\[(\d+)\] = \{([^}]*)\}", src)
    assert int(m.group(1)) == nprim
    pcs = [int(x.strip().rstrip("u")) for x in m.group(2).split(",")]
    assert pcs == [i for i in range(nrec) if prog[i].op == wl.WO_OP_PRIM]
    log = wl.jit_compile_check(src, "gfx950")
    assert log == "", log
    r.close()


def test_literals_round_trip(hostonly):
    """Leaf parameters are emitted as exact fp32 bit patterns (s_mov_b32 immediates)."""
    r = wl.Renderer("lit", max_nodes=8)
    s = r.sphere(0.1)
    h = r.halfspace((0.3, -0.7, 0.2))
    r.union(wl.arg(s, (1.0 / 3.0, 2.0 / 7.0, -1e-7)), wl.arg(h, (0.1, 0.2, 0.3)))
    prog, nrec, _ = r.program()
    src = r.jit_source()
    imms = {int(x, 16) for x in re.findall(r"s_mov_b32 %\d, 0x([0-9a-f]{8})", src)}
    for i in range(nrec):
        if prog[i].op in (wl.WO_LEAF_SPHERE, wl.WO_LEAF_HALFSPACE):
            # axis-aligned half-spaces carry only h as an SGPR constant (s is a literal)
            ks = [3] if prog[i].op == wl.WO_LEAF_HALFSPACE and prog[i].u1 else range(4)
            for k in ks:
                bits = int(np.array(prog[i].f[k], dtype=np.float32).view(np.uint32))
                assert bits in imms, prog[i].f[k]
    assert wl.jit_compile_check(src) == ""
    r.close()


def test_empty_scene_has_no_source(hostonly):
    r = wl.Renderer("e", max_nodes=2)
    assert r.jit_source() is None
    r.close()


def test_member_skip_guards(hostonly, monkeypatch):
    """Members after a primitive's first are guarded by a wave-level emptiness test
    (scene_jit.c member_skip): one guard per later member in each collect pass, none
    with WOLOLO_JIT_MEMBER_SKIP=0.  Exact: a met interval only narrows."""
    guard = "if (__ballot(!(iv.a > iv.b)) != 0ull)"
    r = wl.Renderer("skip", max_nodes=4096)
    scenes.build("csg32", r)
    prog, nrec, _ = r.program()
    src = r.jit_source()
    pair_members = len(re.findall(r"wodev::axis_pair_meet\(", src))  # a pair is one member step
    singles = len(re.findall(r"wodev::(sphere|halfspace|halfspace_axis)_interval\(", src))
    nprims_emitted = 2 * sum(1 for i in range(nrec) if prog[i].op == wl.WO_OP_PRIM)
    assert src.count(guard) == singles + pair_members - nprims_emitted > 0
    monkeypatch.setenv("WOLOLO_JIT_MEMBER_SKIP", "0")
    assert guard not in r.jit_source()
    r.close()
