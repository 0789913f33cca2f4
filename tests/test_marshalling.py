"""Scene marshalling checked independently of the compiler (CPU only).

The GPU-vs-oracle parity tests feed both sides the SAME compiled program
(scene_compile.c) and the same resolved camera, so they cannot see a compiler or
camera bug.  This file closes that gap on the BASELINE scenes themselves:

  * every node call a scene makes through the reference API (renderer.h:28-33,
    node store semantics renderer.c:180-202, 2220-2313; operand placement
    Wo_Node_Argument = rotation then offset, renderer.h:22-27) is recorded, and a
    float64 classifier evaluates the recorded node graph directly -- no use of the
    compiled program;
  * a second classifier evaluates the compiled WoRec program (leaves, convex
    primitives, postfix ops) on the same points; the two must agree everywhere
    except within a thin band around leaf surfaces (fp32 rounding of the leaves);
  * every BOUND record must enclose the part of space where its subtree is inside
    (kernels skip a subtree whose bound a whole wave misses);
  * rays of the scene's own camera, traced by the oracle on the compiled program,
    must hit exactly where the float64 classification of the node graph flips;
  * the look-at camera is restated in double precision and compared with
    wo_renderer_frame_desc.
"""
import math

import numpy as np
import pytest

import pyoracle
from csgrenderer_amd import scenes
from csgrenderer_amd import wololo as wl


class Recorder:
    """Duck-types the Renderer methods scenes.py uses; forwards them to the C library
    and records the node graph, the camera and the leaf materials."""

    def __init__(self, name, max_nodes=4096):
        self.r = wl.Renderer(name, max_nodes=max_nodes)
        self.nodes = []
        self.nonroot = set()
        self.cam = None
        self.leaf_mat = {}
        self.mats = [("lambertian", (0.5, 0.5, 0.5))]

    # ---- nodes ----
    def sphere(self, rad):
        n = self.r.sphere(rad)
        assert n == len(self.nodes)
        self.nodes.append(("s", float(rad)))
        return n

    def halfspace(self, nrm):
        n = self.r.halfspace(nrm)
        assert n == len(self.nodes)
        self.nodes.append(("h", np.array(nrm, dtype=np.float64)))
        return n

    def _binop(self, op, fn, a, b):
        n = fn(a, b)
        assert n == len(self.nodes)
        self.nodes.append((op, a, b))
        self.nonroot.update([a.node, b.node])
        return n

    def union(self, a, b):
        return self._binop("u", self.r.union, a, b)

    def intersection(self, a, b):
        return self._binop("i", self.r.intersection, a, b)

    def difference(self, a, b):
        return self._binop("d", self.r.difference, a, b)

    # ---- materials / camera ----
    def lambertian(self, albedo):
        self.mats.append(("lambertian", tuple(albedo)))
        return self.r.lambertian(albedo)

    def metal(self, albedo, fuzz):
        self.mats.append(("metal", tuple(albedo), fuzz))
        return self.r.metal(albedo, fuzz)

    def dielectric(self, ior):
        self.mats.append(("dielectric", ior))
        return self.r.dielectric(ior)

    def set_material(self, leaf, mat):
        self.leaf_mat[leaf] = mat
        return self.r.set_material(leaf, mat)

    def set_camera(self, look_from, look_at, vup=(0, 1, 0), vfov=90.0, aperture=0.0, focus_dist=1.0):
        self.cam = (look_from, look_at, vup, vfov, aperture, focus_dist)
        return self.r.set_camera(look_from, look_at, vup, vfov, aperture, focus_dist)

    def close(self):
        self.r.close()

    # ---- float64 classification of the recorded graph ----
    @staticmethod
    def _to_local(arg, P):
        q = arg.orientation
        w, x, y, z = q.real, q.imaginary.x, q.imaginary.y, q.imaginary.z
        nq = math.sqrt(w * w + x * x + y * y + z * z)
        w, x, y, z = (1.0, 0.0, 0.0, 0.0) if not nq > 0 else (w / nq, x / nq, y / nq, z / nq)
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        off = np.array([arg.offset.x, arg.offset.y, arg.offset.z])
        return (P - off) @ R  # row-vector form of R^T (p - off)

    def classify(self, node, P):
        """(inside bool[n], distance to the nearest leaf surface met, float[n])."""
        nd = self.nodes[node]
        if nd[0] == "s":
            d = np.sqrt(np.einsum("ij,ij->i", P, P)) - abs(nd[1])
            return d <= 0.0, np.abs(d)
        if nd[0] == "h":
            ln = np.linalg.norm(nd[1])
            if ln == 0:
                return np.ones(len(P), dtype=bool), np.full(len(P), np.inf)
            d = P @ (nd[1] / ln)
            return d <= 0.0, np.abs(d)
        a, da = self.classify(nd[1].node, self._to_local(nd[1], P))
        b, db = self.classify(nd[2].node, self._to_local(nd[2], P))
        v = {"u": a | b, "i": a & b, "d": a & ~b}[nd[0]]
        return v, np.minimum(da, db)

    def scene_classify(self, P):
        inside = np.zeros(len(P), dtype=bool)
        dist = np.full(len(P), np.inf)
        for i in range(len(self.nodes)):
            if i in self.nonroot:
                continue
            v, d = self.classify(i, P)
            inside |= v
            dist = np.minimum(dist, d)
        return inside, dist


def classify_program(prog, nrec, P):
    """Float64 evaluation of the compiled postfix program at points P (n, 3), reading
    the fp32 records as stored.  Returns (inside, violations): violations counts points
    inside a BOUND's subtree but outside its sphere."""
    P = np.asarray(P, dtype=np.float64)
    stack = []
    pending = {}  # end record -> [(centre, R)]
    violations = 0
    pc = 0

    def close_bounds(end):
        nonlocal violations
        for c, R in pending.pop(end, []):
            v = stack[-1]
            d = np.sqrt(((P - c) ** 2).sum(axis=1))
            violations += int((v & (d > R)).sum())

    while pc < nrec:
        rec = prog[pc]
        if rec.op == wl.WO_OP_BOUND:
            pending.setdefault(rec.u0, []).append((np.array(rec.f[:3], dtype=np.float64), float(rec.f[4])))
            pc += 1
            continue
        if rec.op == wl.WO_OP_PRIM:
            v = np.ones(len(P), dtype=bool)
            for m in range(rec.u0):
                L = prog[pc + 1 + m]
                f = np.array(L.f[:4], dtype=np.float64)
                if L.op == wl.WO_LEAF_SPHERE:
                    v &= ((P - f[:3]) ** 2).sum(axis=1) <= f[3]
                else:
                    v &= P @ f[:3] <= f[3]
            stack.append(v)
            pc += 1 + rec.u0
        else:
            b = stack.pop()
            a = stack.pop()
            stack.append({wl.WO_OP_UNION: a | b, wl.WO_OP_INTER: a & b, wl.WO_OP_DIFF: a & ~b,
                          wl.WO_OP_RDIFF: b & ~a}[rec.op])
            pc += 1
        if pc in pending:
            close_bounds(pc)
    assert len(stack) == (1 if nrec else 0)
    return (stack[0] if stack else np.zeros(len(P), dtype=bool)), violations


def _bound_count(prog, nrec):
    return sum(1 for i in range(nrec) if prog[i].op == wl.WO_OP_BOUND)


def _sample_points(rec, rng, n, lo, hi):
    """Uniform points in a box plus points near every sphere leaf's surface (world
    space, from the recorded graph: a sphere operand's centre is its placement)."""
    pts = [rng.uniform(lo, hi, (n, 3))]
    centres = []
    for nd in rec.nodes:
        if nd[0] in "uid":
            for a in (nd[1], nd[2]):
                if rec.nodes[a.node][0] == "s":
                    centres.append((np.array([a.offset.x, a.offset.y, a.offset.z]), rec.nodes[a.node][1]))
    for c, rad in centres:
        if rad > 50:  # a ground sphere: sample its top cap only
            dirs = rng.normal(size=(64, 3)) * np.array([0.01, 1.0, 0.01])
        else:
            dirs = rng.normal(size=(64, 3))
        dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
        radial = rad * (1.0 + rng.uniform(-0.05, 0.05, (64, 1)))
        pts.append(c + dirs * radial)
    return np.concatenate(pts)


# The BASELINE scenes: sample boxes around their geometry
SCENE_BOXES = {
    "csg32": ((-7, -1, -7), (7, 3.5, 7)),
    "rtiow_cover": ((-12, -1, -12), (12, 2.5, 12)),
    "csg256_balanced": ((-6.5, -1, -6.5), (6.5, 3.5, 6.5)),
    "csg256_chain": ((-5.5, -1, -5.5), (5.5, 3.5, 5.5)),
}


def _check_points(rec, prog, nrec, P, band=2e-4):
    want, dist = rec.scene_classify(P)
    got, viol = classify_program(prog, nrec, P)
    assert viol == 0, f"{viol} points inside a bounded subtree lie outside its BOUND sphere"
    bad = (want != got) & (dist > band)
    assert not bad.any(), f"{int(bad.sum())} points classified differently (e.g. {P[bad][:3]})"
    return int(want.sum())


@pytest.mark.parametrize("name", sorted(SCENE_BOXES))
def test_benchmark_scene_compiles_to_the_same_solid(hostonly, name):
    rec = Recorder(name)
    info = scenes.build(name, rec)
    prog, nrec, nprim = rec.r.program()
    assert _bound_count(prog, nrec) > 0
    rng = np.random.default_rng(hash(name) % 2**32)
    lo, hi = SCENE_BOXES[name]
    P = _sample_points(rec, rng, 40000, np.array(lo, float), np.array(hi, float))
    n_in = _check_points(rec, prog, nrec, P)
    assert 0.02 * len(P) < n_in < 0.98 * len(P), (name, n_in)  # the sample sees both sides
    # every leaf is emitted once, carrying the material its node was given
    leaves = [prog[i] for i in range(nrec) if prog[i].op in (wl.WO_LEAF_SPHERE, wl.WO_LEAF_HALFSPACE)]
    assert len(leaves) == info.leaves
    want = sorted(rec.leaf_mat.get(i, 0) for i, nd in enumerate(rec.nodes) if nd[0] in "sh")
    assert sorted(L.u0 for L in leaves) == want
    rec.close()


def _camera_rays(rec, params, n, rng):
    """Primary rays of the recorded camera through pixel centres, restated in double
    (RTIOW positionable camera, no lens)."""
    look_from, look_at, vup, vfov, _, focus = rec.cam
    o = np.array(look_from, float)
    w = o - np.array(look_at, float)
    w /= np.linalg.norm(w)
    u = np.cross(np.array(vup, float), w)
    u /= np.linalg.norm(u)
    v = np.cross(w, u)
    h = math.tan(math.radians(vfov) / 2)
    vh, vw = 2 * h, 2 * h * params.width / params.height
    xs = rng.uniform(0, params.width, n)
    ys = rng.uniform(0, params.height, n)
    dirs = ((xs / params.width - 0.5)[:, None] * vw * u + (0.5 - ys / params.height)[:, None] * vh * v - w)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    return o, dirs


@pytest.mark.parametrize("name", sorted(SCENE_BOXES))
def test_benchmark_scene_rays_hit_where_the_graph_flips(hostonly, name):
    rec = Recorder(name)
    info = scenes.build(name, rec)
    prog, nrec, _ = rec.r.program()
    rng = np.random.default_rng(7 + len(name))
    o, dirs = _camera_rays(rec, info.params(), 150, rng)
    n_hit = n_checked = 0
    for d in dirs:
        of = o.astype(np.float32)
        df = d.astype(np.float32)
        res = pyoracle.trace(prog, nrec, of.tolist(), df.tolist())
        o64, d64 = of.astype(np.float64), df.astype(np.float64)
        if res is None:
            ts = np.linspace(wl.WO_T_MIN + 1e-3, 40.0, 800)
            vals, dist = rec.scene_classify(o64 + ts[:, None] * d64)
            assert (vals[dist > 1e-3] == vals[0]).all(), (name, "missed boundary")
            continue
        t, prim, typ, member, root_after = res
        n_hit += 1
        eps = 2e-4 * max(1.0, t)
        pts = o64 + np.array([t - eps, t + eps])[:, None] * d64
        (before, after), _ = rec.scene_classify(pts)
        if before == after:
            continue  # another boundary within eps
        n_checked += 1
        assert after == bool(root_after), (name, t)
        ts = np.linspace(wl.WO_T_MIN + eps, t - eps, 200)
        vals, dist = rec.scene_classify(o64 + ts[:, None] * d64)
        assert (vals[dist > 1e-4] == before).all(), (name, t, "membership changes before the hit")
    assert n_hit >= 30 and n_checked >= 0.9 * n_hit, (n_hit, n_checked)
    rec.close()


def _big_union_cluster(seed=40):
    """A random union cluster of 60 operands (spheres, lenses, boxes under nested
    rotations, a ground sphere of radius 500) carved by a difference: exercises the surface-area
    split (clusters of >= 16 operands), the giant-operand exclusion and nested BOUNDs."""
    rng = np.random.default_rng(seed)
    rec = Recorder(f"cluster{seed}")
    items = []
    for k in range(48):
        kind = k % 4
        if kind < 2:
            s = rec.sphere(float(rng.uniform(0.2, 0.6)))
            items.append(wl.arg(s, tuple(rng.uniform(-5, 5, 3))))
        elif kind == 2:  # lens: two spheres intersected
            a, b = rec.sphere(0.5), rec.sphere(0.45)
            n = rec.intersection(wl.arg(a), wl.arg(b, (0.3, 0.1, 0.0)))
            q = rng.normal(size=4)
            q /= np.linalg.norm(q)
            items.append(wl.arg(n, tuple(rng.uniform(-5, 5, 3)), wl.Quaternion(q[0], wl.Vec3(*q[1:]))))
        else:  # box: six half-spaces, rotated
            planes = [rec.halfspace(nv) for nv in ((1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1))]
            acc = wl.arg(planes[0], (0.3, 0, 0))
            for p, nv in zip(planes[1:], ((-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1))):
                acc = wl.arg(rec.intersection(acc, wl.arg(p, tuple(0.3 * c for c in nv))))
            # nested placements: the box rotated inside a pair that is rotated again, so
            # the composition order of the two rotations matters
            q1, q2 = rng.normal(size=4), rng.normal(size=4)
            q1 /= np.linalg.norm(q1)
            q2 /= np.linalg.norm(q2)
            knob = rec.sphere(0.15)
            pair = rec.union(wl.arg(acc.node, (0.2, -0.1, 0.3), wl.Quaternion(q1[0], wl.Vec3(*q1[1:]))),
                             wl.arg(knob, (0.5, 0.2, 0.0)))
            items.append(wl.arg(pair, tuple(rng.uniform(-5, 5, 3)), wl.Quaternion(q2[0], wl.Vec3(*q2[1:]))))
    ground = rec.sphere(500.0)
    items.insert(17, wl.arg(ground, (0.0, -505.0, 0.0)))
    order = rng.permutation(len(items))
    items = [items[i] for i in order]
    while len(items) > 1:  # left-deep bracketing, the worst for a BVH until regrouped
        items = [wl.arg(rec.union(items[0], items[1]))] + items[2:]
    carve = rec.sphere(2.0)
    rec.difference(items[0], wl.arg(carve, (1.0, 0.5, -1.0)))
    rec.set_camera((0.0, 3.0, 14.0), (0.0, 0.0, 0.0), (0, 1, 0), 50.0, 0.0, 14.0)
    return rec


def test_union_cluster_sah_and_ground_exclusion(hostonly):
    rec = _big_union_cluster()
    prog, nrec, nprim = rec.r.program()
    assert nprim == 62  # 24 spheres + 12 lenses + 12 boxes with knobs + the ground + the carving sphere
    P = _sample_points(rec, np.random.default_rng(3), 60000, np.array([-6.5, -6.0, -6.5]), np.array([6.5, 6.0, 6.5]))
    _check_points(rec, prog, nrec, P)
    # the ground sphere (r = 500) stays out of the hierarchy: the only giant BOUND is
    # the one around the whole scene (record 0), every bound inside it is small
    radii = [(i, prog[i].f[4]) for i in range(nrec) if prog[i].op == wl.WO_OP_BOUND]
    giant = [i for i, R in radii if R > 50.0]
    assert giant == [0], radii[:4]
    assert max(R for i, R in radii if i != 0) < 10.0
    # bounds nest (a hierarchy, not one flat bound)
    assert _bound_count(prog, nrec) >= 8
    rec.close()


def _camera_restated(cam, W, H):
    """RTIOW camera in double precision, written independently of scene_compile.c."""
    look_from, look_at, vup, vfov, aperture, focus = cam
    o = np.array(look_from, float)
    w = o - np.array(look_at, float)
    w = w / np.linalg.norm(w)
    u = np.cross(np.array(vup, float), w)
    u = u / np.linalg.norm(u)
    v = np.cross(w, u)
    h = math.tan(math.radians(vfov) / 2.0)
    vh = 2.0 * h
    vw = vh * W / H
    horiz = focus * vw * u
    vert = focus * vh * v
    llc = o - horiz / 2 - vert / 2 - focus * w
    return {"origin": o, "lower_left": llc, "horizontal": horiz, "vertical": vert, "u": u, "v": v,
            "lens_radius": np.array([aperture / 2.0])}


CAMERAS = [
    ((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, 0.1, 10.0),        # rtiow_cover
    ((0.0, 4.5, 10.0), (0.0, 0.6, 0.0), (0, 1, 0), 45.0, 0.0, 10.0),  # csg32
    ((0.0, 6.0, 13.0), (0.0, 0.8, 0.0), (0, 1, 0), 45.0, 0.0, 13.0),  # csg256
    ((-3.0, 1.5, -2.0), (4.0, -0.5, 7.0), (0.2, 1.0, -0.1), 73.0, 0.5, 3.7),
]


@pytest.mark.parametrize("cam", CAMERAS)
@pytest.mark.parametrize("size", [(1920, 1080), (3840, 2160), (77, 43)])
def test_camera_matches_a_double_restatement(hostonly, cam, size):
    r = wl.Renderer("cam", max_nodes=4)
    r.set_camera(*cam)
    W, H = size
    fr = r.frame_desc(wl.render_params(W, H, spp=1, mode=wl.MODE_PATHTRACE))
    want = _camera_restated(cam, W, H)
    for field, ref in want.items():
        got = np.atleast_1d(np.array(getattr(fr.cam, field), dtype=np.float32)).astype(np.float64)
        # one fp32 rounding of the double value (plus a few double ulps of order)
        tol = np.abs(ref) * 2.0 ** -23 + 1e-12
        assert np.all(np.abs(got - ref) <= tol), (field, got, ref)
    assert fr.inv_width == np.float32(1.0 / W) and fr.inv_height == np.float32(1.0 / H)
    r.close()
