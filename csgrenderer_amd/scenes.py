"""Benchmark / parity scenes of BASELINE.json, built through the wololo node API.

Every scene is constructed only with the reference's node calls
(``wo_renderer_add_{sphere,infinite_planar_partition,union_of,intersection_of,
difference_of}_node``, renderer.h:28-33) plus the material/camera extensions, so
the same scene can be built from C.  Scene randomness uses PCG32 (O'Neill's
pcg32_random_r, 64-bit LCG state, XSH-RR output) seeded as SURVEY.md §8(d) says:
C2 0x5EED, C3 32, C5 256.

Configs:
  C1 sphere256   the reference shader, 256x256, 1 spp (no nodes needed)
  C2 rtiow_cover RTIOW final scene, ~480 spheres as a balanced union tree
  C3 csg32       32 leaves (20 spheres + 2 six-plane boxes), 31 binops, 63 nodes
  C4 csg32_4k    C3 at 3840x2160, 256 spp (8-GPU row tiles)
  C5 csg256      128 sphere leaves, 255 nodes: balanced tree or left-deep chain
"""
from __future__ import annotations

import math
from dataclasses import dataclass

from .wololo import (MODE_PATHTRACE, MODE_UBERSHADER_RT1, Renderer, arg, render_params)


class Pcg32:
    """pcg32_random_r with the default stream increment (seq 0x5851F42D... style)."""

    MUL = 6364136223846793005
    MASK = (1 << 64) - 1

    def __init__(self, seed: int, seq: int = 0xDA3E39CB94B95BDB):
        self.state = 0
        self.inc = ((seq << 1) | 1) & self.MASK
        self.next_u32()
        self.state = (self.state + seed) & self.MASK
        self.next_u32()

    def next_u32(self) -> int:
        old = self.state
        self.state = (old * self.MUL + self.inc) & self.MASK
        xorshifted = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xorshifted >> rot) | (xorshifted << ((-rot) & 31))) & 0xFFFFFFFF

    def random(self) -> float:
        """Uniform double in [0, 1) (32 random bits)."""
        return self.next_u32() / 4294967296.0

    def uniform(self, lo: float, hi: float) -> float:
        return lo + (hi - lo) * self.random()


@dataclass
class SceneInfo:
    name: str
    spheres: int
    halfspaces: int
    binops: int
    width: int
    height: int
    spp: int
    max_depth: int
    mode: int = MODE_PATHTRACE
    shape: str = ""  # the CSG tree's shape, for the bench line's workload label

    @property
    def leaves(self) -> int:
        return self.spheres + self.halfspaces

    @property
    def flop_per_segment(self) -> int:
        """30 per ray-sphere, 12 per ray-half-space, 4 per binop, 40 shading."""
        return 30 * self.spheres + 12 * self.halfspaces + 4 * self.binops + 40

    def params(self, **over):
        kw = dict(width=self.width, height=self.height, spp=self.spp, max_depth=self.max_depth, mode=self.mode)
        kw.update(over)
        return render_params(**kw)


def _balanced(r: Renderer, items, ops):
    """items: list of (node, offset).  Returns (node, offset) of a balanced tree whose
    internal nodes take their operator from ops() in creation order."""
    if len(items) == 1:
        return items[0]
    h = len(items) // 2
    ln, lo = _balanced(r, items[:h], ops)
    rn, ro = _balanced(r, items[h:], ops)
    op = ops()
    n = {"u": r.union, "d": r.difference, "i": r.intersection}[op](arg(ln, lo), arg(rn, ro))
    return n, (0.0, 0.0, 0.0)


def _cycle(seq):
    state = {"i": 0}

    def nxt():
        v = seq[state["i"] % len(seq)]
        state["i"] += 1
        return v

    return nxt


def _root(r: Renderer, item):
    """A lone placed leaf cannot be a root (placement lives on binop operands):
    wrap it as a union with itself."""
    n, off = item
    if off == (0.0, 0.0, 0.0):
        return n
    return r.union(arg(n, off), arg(n, off))


def _random_material(r: Renderer, rng: Pcg32):
    choose = rng.random()
    if choose < 0.8:
        return r.lambertian((rng.random() * rng.random(), rng.random() * rng.random(), rng.random() * rng.random()))
    if choose < 0.95:
        return r.metal((rng.uniform(0.5, 1), rng.uniform(0.5, 1), rng.uniform(0.5, 1)), rng.uniform(0, 0.5))
    return r.dielectric(1.5)


# ---------------------------------------------------------------------------------------------
def sphere256() -> SceneInfo:
    """C1: the reference path itself -- no scene nodes (ubershader1.frag ignores them)."""
    return SceneInfo("sphere256", spheres=1, halfspaces=0, binops=0, width=256, height=256, spp=1, max_depth=1,
                     mode=MODE_UBERSHADER_RT1)


def build_rtiow_cover(r: Renderer, seed: int = 0x5EED) -> SceneInfo:
    """C2: Ray Tracing in One Weekend's final scene (book 1, §13)."""
    rng = Pcg32(seed)
    items = []
    ground = r.sphere(1000.0)
    r.set_material(ground, r.lambertian((0.5, 0.5, 0.5)))
    items.append((ground, (0.0, -1000.0, 0.0)))
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose = rng.random()
            cx, cz = a + 0.9 * rng.random(), b + 0.9 * rng.random()
            if math.sqrt((cx - 4.0) ** 2 + 0.0 + cz ** 2) <= 0.9:
                continue
            if choose < 0.8:
                m = r.lambertian((rng.random() * rng.random(), rng.random() * rng.random(),
                                  rng.random() * rng.random()))
            elif choose < 0.95:
                m = r.metal((rng.uniform(0.5, 1), rng.uniform(0.5, 1), rng.uniform(0.5, 1)), rng.uniform(0, 0.5))
            else:
                m = r.dielectric(1.5)
            s = r.sphere(0.2)
            r.set_material(s, m)
            items.append((s, (cx, 0.2, cz)))
    big = [((0.0, 1.0, 0.0), r.dielectric(1.5)), ((-4.0, 1.0, 0.0), r.lambertian((0.4, 0.2, 0.1))),
           ((4.0, 1.0, 0.0), r.metal((0.7, 0.6, 0.5), 0.0))]
    for c, m in big:
        s = r.sphere(1.0)
        r.set_material(s, m)
        items.append((s, c))
    n = len(items)
    _root(r, _balanced(r, items, _cycle("u")))
    r.set_camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, 0.1, 10.0)
    return SceneInfo("rtiow_cover", spheres=n, halfspaces=0, binops=n - 1, width=1920, height=1080, spp=64,
                     max_depth=8)


def _box(r: Renderer, center, half: float):
    return _box_extents(r, center, (half, half, half))


def _box_extents(r: Renderer, center, half):
    """Axis-aligned box as a 6-half-space intersection chain (planes placed by offset)."""
    normals = [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)]
    planes = [(r.halfspace(n), tuple(c + h * k for c, h, k in zip(center, half, n))) for n in normals]
    node, off = planes[0]
    acc = None
    for p, poff in planes[1:]:
        if acc is None:
            acc = r.intersection(arg(node, off), arg(p, poff))
        else:
            acc = r.intersection(arg(acc), arg(p, poff))
    return acc, [p for p, _ in planes]


def _overlapping_pairs(r: Renderer, rng: Pcg32, n_pairs: int, lo, hi, rmin: float, rmax: float, ops):
    """n_pairs overlapping sphere pairs; pair k is combined with ops() so the CSG op
    actually cuts (a lens, a bitten sphere or a blob).  Returns placed items."""
    items = []
    for _ in range(n_pairs):
        ra = rng.uniform(rmin, rmax)
        rb = rng.uniform(rmin, rmax)
        ca = tuple(rng.uniform(a, b) for a, b in zip(lo, hi))
        # second centre at 0.6..0.9 of the radius sum in a random direction
        th, ph = rng.uniform(0, 2 * math.pi), math.acos(rng.uniform(-1, 1))
        dist = rng.uniform(0.6, 0.9) * (ra + rb) * 0.75
        cb = (ca[0] + dist * math.sin(ph) * math.cos(th), ca[1] + dist * math.cos(ph),
              ca[2] + dist * math.sin(ph) * math.sin(th))
        sa, sb = r.sphere(ra), r.sphere(rb)
        r.set_material(sa, _random_material(r, rng))
        r.set_material(sb, _random_material(r, rng))
        op = {"u": r.union, "d": r.difference, "i": r.intersection}[ops()]
        items.append((op(arg(sa, ca), arg(sb, cb)), (0.0, 0.0, 0.0)))
    return items


def build_csg32(r: Renderer, seed: int = 32, width=1920, height=1080, spp=64, union_only=False) -> SceneInfo:
    """C3: 32 leaves (20 spheres + 12 half-spaces), 31 binops, 63 nodes.

    Box A is a 12 x 0.5 x 12 floor slab (y in [-0.5, 0]) minus sphere0 (a crater);
    box B a 1.5-unit cube intersected with sphere1 (a rounded cube); the other 18
    spheres form 9 overlapping pairs whose ops cycle union / difference /
    intersection, joined by a balanced union.  (SURVEY.md §8(d) sketches C3 with two
    small boxes; the slab keeps the leaf/binop counts and gives the paths a floor
    to bounce off.)"""
    rng = Pcg32(seed)
    slab, planes_a = _box_extents(r, (0.0, -0.25, 0.0), (6.0, 0.25, 6.0))
    cube, planes_b = _box(r, (-2.0, 0.75, 0.0), 0.75)
    ma, mb = r.lambertian((0.5, 0.5, 0.5)), r.metal((0.8, 0.8, 0.9), 0.05)
    for p in planes_a:
        r.set_material(p, ma)
    for p in planes_b:
        r.set_material(p, mb)
    s0, s1 = r.sphere(1.2), r.sphere(1.0)
    r.set_material(s0, r.lambertian((0.7, 0.3, 0.2)))
    r.set_material(s1, r.metal((0.9, 0.8, 0.5), 0.1))
    crater = (r.union if union_only else r.difference)(arg(slab), arg(s0, (2.5, 0.3, 1.5)))
    rounded = r.intersection(arg(cube), arg(s1, (-2.0, 0.75, 0.0)))
    pairs = _overlapping_pairs(r, rng, 9, (-4.0, 0.5, -4.0), (4.0, 2.0, 4.0), 0.3, 0.8,
                               _cycle("uui" if union_only else "udi"))
    rest, roff = _balanced(r, pairs, _cycle("u"))
    objs = r.union(arg(crater), arg(rounded))
    r.union(arg(objs), arg(rest, roff))
    r.set_camera((0.0, 4.5, 10.0), (0.0, 0.6, 0.0), (0, 1, 0), 45.0, 0.0, 10.0)
    return SceneInfo("csg32_union" if union_only else "csg32", spheres=20, halfspaces=12, binops=31, width=width, height=height, spp=spp,
                     max_depth=8,
                     shape="root union of 14 terms of <= 2 literals" if not union_only else "union of primitives")


class NestedShape:
    """Host mirror of a csg32_nested subtree, for the non-emptiness check
    (tests/test_scenes.py): leaves are spheres (centre, radius) or axis boxes
    (centre, half extents); binops carry their operator."""

    def __init__(self, op, a=None, b=None, centre=None, size=None):
        self.op, self.a, self.b, self.centre, self.size = op, a, b, centre, size

    def contains(self, pts):
        """Membership of an (n, 3) float64 array of points."""
        import numpy as np
        if self.op == "sphere":
            return ((pts - np.asarray(self.centre)) ** 2).sum(axis=1) <= self.size ** 2
        if self.op == "box":
            return (np.abs(pts - np.asarray(self.centre)) <= np.asarray(self.size)).all(axis=1)
        a, b = self.a.contains(pts), self.b.contains(pts)
        return {"u": a | b, "i": a & b, "d": a & ~b}[self.op]

    def nodes(self, depth=0):
        """(depth, node) of every binop, pre-order."""
        if self.a is None:
            return []
        return [(depth, self)] + self.a.nodes(depth + 1) + self.b.nodes(depth + 1)


# csg32_nested: the operator of the j-th binop (left to right) at depth d of the
# balanced tree; the root subtracts, and every level below has both
# intersections and differences (and unions)
_NESTED_OPS = "dui"


def build_csg32_nested(r: Renderer, seed: int = 3235, width=1920, height=1080, spp=64, mirror=None,
                       items: int = 22, boxes=(6, 17)) -> SceneInfo:
    """C3 as SURVEY.md §8(d) wrote it: 32 leaves (20 spheres + 12 half-spaces forming two
    6-plane boxes) in ONE balanced tree with intersections and differences at every
    level (31 binops, 63 nodes) -- unlike csg32, whose root is a union of small terms
    that the specialised kernel's union count is built for.

    Placement makes every operation count: a subtree is built to fill a ball (centre,
    R); a union puts its operands side by side, an intersection overlaps them by most
    of their size, a difference bites a smaller operand out of the side of a larger
    one.  tests/test_scenes.py checks on sampled points that every intersection and
    every difference of the built tree is non-empty and that every difference removes
    something.  `mirror` (a list) receives the tree's NestedShape.

    `items` / `boxes`: the same construction over more leaves (csg360_nested: 337
    spheres and 23 boxes, 474 binops, 309 primitives -- the > 256-primitive general tree)."""
    rng = Pcg32(seed)
    n_items = items  # csg32_nested: 20 spheres + 2 boxes (a box is a chain of 6 half-space intersections)
    box_at = set(boxes)
    pos_at_depth = {}
    leaf_no = [0]

    def unit():
        th, ph = rng.uniform(0, 2 * math.pi), math.acos(rng.uniform(-0.6, 0.6))
        return (math.sin(ph) * math.cos(th), math.cos(ph), math.sin(ph) * math.sin(th))

    def add(c, k, d):
        return tuple(ci + k * di for ci, di in zip(c, d))

    def build(n, centre, rad, depth):
        if n == 1:
            k = leaf_no[0]
            leaf_no[0] += 1
            if k in box_at:
                half = (0.8 * rad, 0.55 * rad, 0.8 * rad)
                node, planes = _box_extents(r, centre, half)
                m = r.metal((0.8, 0.85, 0.9), 0.05) if k % 2 == 0 else r.lambertian((0.3, 0.5, 0.7))
                for pl in planes:
                    r.set_material(pl, m)
                return (node, (0.0, 0.0, 0.0)), NestedShape("box", centre=centre, size=half)
            sph = r.sphere(rad)
            r.set_material(sph, _random_material(r, rng))
            return (sph, centre), NestedShape("sphere", centre=centre, size=rad)
        j = pos_at_depth.get(depth, 0)
        pos_at_depth[depth] = j + 1
        op = _NESTED_OPS[(depth + j) % 3]
        d = unit()
        nl = n // 2
        if op == "u":
            (la, ma), (lb, mb) = build(nl, add(centre, -0.45 * rad, d), 0.7 * rad, depth + 1), \
                build(n - nl, add(centre, 0.45 * rad, d), 0.7 * rad, depth + 1)
        elif op == "i":
            (la, ma), (lb, mb) = build(nl, add(centre, -0.15 * rad, d), 1.0 * rad, depth + 1), \
                build(n - nl, add(centre, 0.15 * rad, d), 1.0 * rad, depth + 1)
        else:
            (la, ma), (lb, mb) = build(nl, centre, 1.0 * rad, depth + 1), \
                build(n - nl, add(centre, 0.6 * rad, d), 0.75 * rad, depth + 1)
        node = {"u": r.union, "d": r.difference, "i": r.intersection}[op](arg(*la), arg(*lb))
        return (node, (0.0, 0.0, 0.0)), NestedShape(op, ma, mb)

    (root, _), shape = build(n_items, (0.0, 1.6, 0.0), 2.6, 0)
    if mirror is not None:
        mirror.append(shape)
    r.set_camera((0.0, 2.4, 6.0), (0.0, 1.4, 0.0), (0, 1, 0), 38.0, 0.0, 6.0)
    nb = len(box_at)
    name = "csg32_nested" if n_items == 22 else f"csg{n_items}_nested"
    return SceneInfo(name, spheres=n_items - nb, halfspaces=6 * nb, binops=n_items - 1 + 5 * nb, width=width,
                     height=height, spp=spp, max_depth=8,
                     shape="one balanced tree, intersections and differences at every level")


def build_csg256(r: Renderer, seed: int = 256, shape: str = "balanced", width=1920, height=1080,
                 spp=64, union_only=False, pairs: int = 63) -> SceneInfo:
    """C5: 128 sphere leaves, 127 binops (255 nodes), leaf 0 an RTIOW-style ground
    sphere (r = 1000).
      balanced: 63 overlapping pairs (ops cycle u/d/i) + ground + 1 sphere, joined
                by a balanced union;
      chain:    a left-deep chain of depth 127 starting from the ground, ops cycling
                u/u/d, so later spheres carve earlier ones and the ground."""
    rng = Pcg32(seed)
    ground = r.sphere(1000.0)
    r.set_material(ground, r.lambertian((0.5, 0.5, 0.5)))
    gitem = (ground, (0.0, -1000.0, 0.0))
    if shape == "balanced":
        items = [gitem] + _overlapping_pairs(r, rng, pairs, (-5.0, 0.3, -5.0), (5.0, 2.5, 5.0), 0.25, 0.6,
                                               _cycle("uui" if union_only else "udi"))
        s = r.sphere(1.0)
        r.set_material(s, r.dielectric(1.5))
        items.append((s, (0.0, 1.0, 0.0)))
        _root(r, _balanced(r, items, _cycle("u")))
    elif shape == "chain":
        ops = _cycle("uud")
        n, off = gitem
        acc = None
        for _ in range(127):
            rad = rng.uniform(0.3, 0.7)
            c = (rng.uniform(-4, 4), rng.uniform(0.0, 2.0), rng.uniform(-4, 4))
            s = r.sphere(rad)
            r.set_material(s, _random_material(r, rng))
            op = {"u": r.union, "d": r.difference}[ops()]
            acc = op(arg(n, off), arg(s, c)) if acc is None else op(arg(acc), arg(s, c))
    else:
        raise ValueError(shape)
    r.set_camera((0.0, 6.0, 13.0), (0.0, 0.8, 0.0), (0, 1, 0), 45.0, 0.0, 13.0)
    leaves = 2 * pairs + 2 if shape == "balanced" else 128
    name = f"csg256_{shape}" if leaves == 128 else f"csg{leaves}_{shape}"
    return SceneInfo(name + ("_union" if union_only else ""), spheres=leaves, halfspaces=0, binops=leaves - 1, width=width,
                     height=height, spp=spp, max_depth=8)


SCENES = {
    "rtiow_cover": build_rtiow_cover,
    "csg32": build_csg32,
    "csg32_nested": build_csg32_nested,
    # csg32's geometry with the differences made unions (an A/B scene for the
    # union-only lane tracer; not a BASELINE config)
    "csg32_union": lambda r, **k: build_csg32(r, union_only=True, **k),
    "csg256_balanced_union": lambda r, **k: build_csg256(r, shape="balanced", union_only=True, **k),
    "csg256_balanced": lambda r, **k: build_csg256(r, shape="balanced", **k),
    "csg256_chain": lambda r, **k: build_csg256(r, shape="chain", **k),
    # more than WOLOLO_JIT_MAX_PRIMS primitives and not union-only: the interpreter's
    # scene (512 sphere leaves: 255 overlapping pairs + ground + glass ball, 427
    # primitives) -- not a BASELINE config, the measure of the >256-primitive path
    "csg512_balanced": lambda r, **k: build_csg256(r, shape="balanced", pairs=255, **k),
    # csg32_nested's construction over 360 items (337 spheres, 23 boxes: 475 leaves, 309
    # primitives): a general tree (intersections and differences at every level) of more
    # than 256 primitives -- not a BASELINE config, the measure of that path
    "csg360_nested": lambda r, **k: build_csg32_nested(r, items=360, boxes=range(7, 360, 16), **k),
}


def build(name: str, r: Renderer, **kw) -> SceneInfo:
    return SCENES[name](r, **kw)
