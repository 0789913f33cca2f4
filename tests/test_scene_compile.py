"""Scene compiler (csrc/scene_compile.c) checked independently (CPU only).

The node tables the reference keeps on the host (renderer.c:180-202) never reach
its GPU, so the compile step defines the scene semantics.  Here a Python shadow of
the node tables classifies points in float64 directly (recursive point-in-CSG with
each operand's rotation+offset inverted), with no use of the compiled program; the
oracle's hits on random rays must be exactly where that classification changes.
"""
import math

import numpy as np
import pytest

import pyoracle
from csgrenderer_amd import scenes
from csgrenderer_amd import wololo as wl


class Shadow:
    """Records nodes as they are added through the C API."""

    def __init__(self, r: wl.Renderer):
        self.r = r
        self.nodes = []
        self.nonroot = set()

    def sphere(self, rad):
        n = self.r.sphere(rad)
        self.nodes.append(("s", rad))
        return n

    def halfspace(self, nrm):
        n = self.r.halfspace(nrm)
        self.nodes.append(("h", np.array(nrm, dtype=np.float64)))
        return n

    def binop(self, op, a, b):
        fn = {"u": self.r.union, "i": self.r.intersection, "d": self.r.difference}[op]
        n = fn(a, b)
        self.nodes.append((op, a, b))
        self.nonroot.update([a.node, b.node])
        return n

    # ---- float64 point classification ----
    @staticmethod
    def _to_local(arg, p):
        q = arg.orientation
        w, x, y, z = q.real, q.imaginary.x, q.imaginary.y, q.imaginary.z
        nq = math.sqrt(w * w + x * x + y * y + z * z)
        w, x, y, z = (1.0, 0.0, 0.0, 0.0) if nq == 0 else (w / nq, x / nq, y / nq, z / nq)
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        off = np.array([arg.offset.x, arg.offset.y, arg.offset.z])
        return R.T @ (p - off)

    def inside(self, node, p):
        nd = self.nodes[node]
        if nd[0] == "s":
            return float(np.dot(p, p)) <= abs(nd[1]) ** 2
        if nd[0] == "h":
            n = nd[1]
            ln = np.linalg.norm(n)
            return True if ln == 0 else float(np.dot(n / ln, p)) <= 0.0
        a = self.inside(nd[1].node, self._to_local(nd[1], p))
        b = self.inside(nd[2].node, self._to_local(nd[2], p))
        return {"u": a or b, "i": a and b, "d": a and not b}[nd[0]]

    def scene_inside(self, p):
        return any(self.inside(i, p) for i in range(len(self.nodes)) if i not in self.nonroot)


def _rand_quat(rng):
    v = rng.normal(size=4)
    v /= np.linalg.norm(v)
    return wl.Quaternion(v[0], wl.Vec3(v[1], v[2], v[3]))


def _random_scene(seed, n_leaves=10, axis=False):
    """axis=True: half-space normals are +-e_a and operands are only translated, so
    the compiled leaves are axis-aligned (u1 != 0) and take the reciprocal path."""
    rng = np.random.default_rng(seed)
    r = wl.Renderer(f"rand{seed}", max_nodes=256)
    sh = Shadow(r)
    pool = []
    for _ in range(n_leaves):
        if rng.random() < 0.7:
            pool.append(sh.sphere(rng.uniform(0.4, 1.2)))
        else:
            nrm = np.eye(3)[rng.integers(3)] * rng.choice([-1.0, 1.0]) if axis else rng.normal(size=3)
            pool.append(sh.halfspace(nrm))
    while len(pool) > 1:
        i, j = rng.choice(len(pool), 2, replace=False)
        a, b = pool[i], pool[j]
        op = rng.choice(["u", "i", "d"], p=[0.45, 0.3, 0.25])
        mk = lambda n: wl.arg(n, tuple(rng.uniform(-1.0, 1.0, 3)),
                              _rand_quat(rng) if rng.random() < 0.5 and not axis else None)
        n = sh.binop(op, mk(a), mk(b))
        pool = [x for k, x in enumerate(pool) if k not in (i, j)] + [n]
    return r, sh, rng


def _program_checks(prog, nrec, nprim):
    sp, maxsp, ords, pc = 0, 0, [], 0
    bounds = []
    while pc < nrec:
        op = prog[pc].op
        if op == wl.WO_OP_PRIM:
            ords.append(prog[pc].u1)
            for m in range(prog[pc].u0):
                L = prog[pc + 1 + m]
                assert L.op in (wl.WO_LEAF_SPHERE, wl.WO_LEAF_HALFSPACE)
                if L.op == wl.WO_LEAF_HALFSPACE:
                    # u1 = 1 + a exactly when the normal is +-e_a (wo_scene.h)
                    f = list(L.f[:3])
                    axes = [a for a in range(3) if abs(f[a]) == 1.0 and f[(a + 1) % 3] == 0.0
                            and f[(a + 2) % 3] == 0.0]
                    assert L.u1 == (1 + axes[0] if axes else 0), (f, L.u1)
            sp += 1
            pc += 1 + prog[pc].u0
        elif op == wl.WO_OP_BOUND:
            assert pc < prog[pc].u0 <= nrec
            bounds.append((pc, prog[pc].u0))
            pc += 1
        else:
            assert op in (wl.WO_OP_UNION, wl.WO_OP_INTER, wl.WO_OP_DIFF, wl.WO_OP_RDIFF)
            assert sp >= 2
            sp -= 1
            pc += 1
        maxsp = max(maxsp, sp)
    assert ords == list(range(nprim))
    assert (sp == 1) if nprim else (sp == 0)
    assert maxsp <= 31
    # a BOUND's skip target ends a complete subtree: evaluating [pc+1, skip) leaves one value
    for b, skip in bounds:
        depth, k = 0, b + 1
        while k < skip:
            op = prog[k].op
            if op == wl.WO_OP_PRIM:
                depth += 1
                k += 1 + prog[k].u0
            elif op == wl.WO_OP_BOUND:
                k += 1
            else:
                depth -= 1
                k += 1
        assert k == skip and depth == 1
        # u1 = leaves in the bounded subtree (kernels skip testing small BOUNDs)
        nleaf = sum(1 for j in range(b + 1, skip) if prog[j].op in (wl.WO_LEAF_SPHERE, wl.WO_LEAF_HALFSPACE))
        assert prog[b].u1 == nleaf
    return maxsp


@pytest.mark.parametrize("name", ["csg32", "rtiow_cover", "csg256_balanced", "csg256_chain"])
def test_benchmark_scene_programs(hostonly, name):
    r = wl.Renderer(name, max_nodes=4096)
    info = scenes.build(name, r)
    prog, nrec, nprim = r.program()
    depth = _program_checks(prog, nrec, nprim)
    nleaf = sum(1 for i in range(nrec) if prog[i].op in (wl.WO_LEAF_SPHERE, wl.WO_LEAF_HALFSPACE))
    assert nleaf == info.leaves
    assert depth <= math.ceil(math.log2(max(nprim, 2))) + 1  # Sethi-Ullman bound
    r.close()


def test_csg32_counts(hostonly):
    r = wl.Renderer("c", max_nodes=4096)
    info = scenes.build("csg32", r)
    assert (info.spheres, info.halfspaces, info.binops) == (20, 12, 31)
    assert r.lib.wo_renderer_node_count(r.ptr) == 63
    r.close()


def test_bounds_enclose_their_spheres(hostonly):
    r = wl.Renderer("b", max_nodes=4096)
    scenes.build("rtiow_cover", r)
    prog, nrec, _ = r.program()
    checked = 0
    for b in range(nrec):
        if prog[b].op != wl.WO_OP_BOUND:
            continue
        c = np.array(prog[b].f[:3], dtype=np.float64)
        R = float(prog[b].f[4])
        assert R * R <= float(prog[b].f[3]) * (1 + 1e-6)
        for k in range(b + 1, prog[b].u0):
            if prog[k].op == wl.WO_LEAF_SPHERE:
                cc = np.array(prog[k].f[:3], dtype=np.float64)
                rad = math.sqrt(prog[k].f[3])
                assert np.linalg.norm(cc - c) + rad <= R * (1 + 1e-6)
                checked += 1
    assert checked > 480


@pytest.mark.parametrize("seed,axis", [(s, False) for s in range(12)] + [(s, True) for s in range(100, 106)])
def test_random_scenes_hits_match_float64_classifier(hostonly, seed, axis):
    r, sh, rng = _random_scene(seed, axis=axis)
    prog, nrec, nprim = r.program()
    _program_checks(prog, nrec, nprim)
    if axis:
        assert all(prog[i].u1 != 0 for i in range(nrec) if prog[i].op == wl.WO_LEAF_HALFSPACE)
    n_hit = n_checked = 0
    for _ in range(60):
        o = rng.uniform(-4, 4, 3) * np.array([1, 1, 1]) + np.array([0, 0, 6.0])
        tgt = rng.uniform(-1.5, 1.5, 3)
        d = tgt - o
        d = (d / np.linalg.norm(d)).astype(np.float32)
        o = o.astype(np.float32)
        of, df = o.astype(np.float64), d.astype(np.float64)
        res = pyoracle.trace(prog, nrec, o.tolist(), d.tolist())
        tmin = wl.WO_T_MIN
        if res is None:
            # no boundary crossing: the classification is constant along the ray
            ts = np.linspace(tmin + 1e-3, 30.0, 400)
            vals = [sh.scene_inside(of + t * df) for t in ts]
            # a sampled change of membership means the oracle missed a boundary
            assert len(set(vals)) == 1, (seed, "missed boundary")
            continue
        t, prim, typ, member, root_after = res
        n_hit += 1
        eps = 2e-4 * max(1.0, t)
        before = sh.scene_inside(of + (t - eps) * df)
        after = sh.scene_inside(of + (t + eps) * df)
        if before == after:
            continue  # another boundary within eps (numerically ambiguous); skip
        n_checked += 1
        assert after == bool(root_after), (seed, t)
        # nothing changes between tmin and the hit
        ts = np.linspace(tmin + eps, t - eps, 64)
        first = sh.scene_inside(of + ts[0] * df)
        assert first == before
        assert all(sh.scene_inside(of + s * df) == first for s in ts), (seed, t)
    assert n_checked >= n_hit * 0.8
    # rays aimed at points the float64 classifier puts inside the solid must report a
    # boundary no later than the point (covers trees whose solid is tiny or empty)
    pts = np.random.default_rng(seed).uniform(-4, 4, (3000, 3))
    inside_pts = [p for p in pts if sh.scene_inside(p)][:20]
    for p in inside_pts:
        o = np.array([0.0, 0.5, 9.0]) + rng.uniform(-1, 1, 3)
        if sh.scene_inside(o):
            continue
        d = p - o
        dist = np.linalg.norm(d)
        d = (d / dist).astype(np.float32)
        res = pyoracle.trace(prog, nrec, o.astype(np.float32).tolist(), d.tolist())
        assert res is not None and res[0] <= dist * (1 + 1e-4) + 1e-4, (seed, p, res)
    r.close()


def test_deep_difference_chain_fails_cleanly(hostonly):
    """A user-built chain deeper than the compiler's recursion limit (8192 levels) is an
    error, not a native stack overflow; a 4000-deep chain compiles."""
    for depth, ok in [(4000, True), (9000, False)]:
        r = wl.Renderer(f"chain{depth}", max_nodes=2 * depth + 4)
        acc = r.sphere(1.0)
        for k in range(depth):
            s = r.sphere(0.1)
            acc = r.difference(wl.arg(acc), wl.arg(s, (0.0, 0.0, 0.001 * k)))
        if ok:
            assert r.compile() > 0
        else:
            with pytest.raises(wl.WololoError, match="too deep"):
                r.compile()
        r.close()


def test_sphere_leaf_out_of_fp32_range_fails_cleanly(hostonly):
    """A sphere whose radius^2 or centre is not a finite fp32 value is refused by the
    compiler: the kernels' square root of the discriminant (sqrt_cr, rsq + one Markstein
    step) is exact for every finite argument but gives NaN at +inf, and a
    finite r^2 with a finite ray keeps the discriminant below +inf.  1e19 (r^2 = 1e38)
    still compiles."""
    for rad, off, ok in [(1e19, 0.0, True), (2e19, 0.0, False), (1.0, 1e39, False)]:
        r = wl.Renderer("big", max_nodes=8)
        s, t = r.sphere(rad), r.sphere(1.0)
        r.union(wl.arg(s, (off, 0.0, 0.0)), wl.arg(t))
        if ok:
            assert r.compile() > 0
        else:
            with pytest.raises(wl.WololoError, match="fp32 range"):
                r.compile()
        r.close()
