"""GPU parity: HIP kernels (through the C-ABI of libwololo.so) vs the CPU oracle.

Bar: bit-exact (max |delta| == 0) for every comparison below -- both sides are
IEEE fp32 with the same op order, correctly rounded div/sqrt and no contraction.
The north_star tolerance (1e-4 max per channel) is asserted as well so a
failure message shows which bar broke.
"""
import json
import os
import time

import numpy as np
import pytest

import pyoracle
from csgrenderer_amd import scenes
from csgrenderer_amd import wololo as wl

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-4  # north_star: max per-channel |delta| < 1e-4


def _cmp(gpu, ref, what):
    gpu = np.asarray(gpu, dtype=np.float32)
    ref = np.asarray(ref, dtype=np.float32)
    assert gpu.shape == ref.shape, what
    both_nan = np.isnan(gpu) & np.isnan(ref)
    d = np.where(both_nan, 0.0, np.abs(gpu.astype(np.float64) - ref.astype(np.float64)))
    mx = float(np.nanmax(d)) if d.size else 0.0
    nbad = int((d > 0).sum())
    assert mx < TOL, f"{what}: max |delta| {mx} >= {TOL} ({nbad} values differ)"
    assert nbad == 0, f"{what}: not bit-exact ({nbad} values differ, max {mx})"


@pytest.fixture(scope="module")
def empty_renderer():
    r = wl.Renderer("uber", max_nodes=8)
    yield r
    r.close()


@pytest.mark.parametrize("w,h", [(256, 256), (1280, 720), (1920, 1080), (3840, 2160), (17, 5), (1, 1)])
@pytest.mark.parametrize("t", [0.0, 1.0, 0.37, 2.5])
def test_ubershader_bitexact(empty_renderer, w, h, t):
    img = empty_renderer.render(wl.render_params(w, h, time_sec=t, mode=wl.MODE_UBERSHADER_RT1))
    ref = pyoracle.ubershader_frame(w, h, t, 0)
    _cmp(img, ref, f"ubershader {w}x{h} t={t}")


def test_debug_view_bitexact(empty_renderer):
    img = empty_renderer.render(wl.render_params(640, 360, mode=wl.MODE_DEBUG_ST))
    ref = pyoracle.ubershader_frame(640, 360, 0.0, 1)
    _cmp(img, ref, "ep_debug_view_1")


def test_ubershader_kats_on_gpu(empty_renderer):
    kats = json.load(open(os.path.join(GOLD, "ubershader_kats.json")))
    cache = {}
    for k in kats["pixels"]:
        key = (k["w"], k["h"], k["t"])
        if key not in cache:
            cache[key] = empty_renderer.render(wl.render_params(k["w"], k["h"], time_sec=k["t"]))
        got = cache[key][k["y"], k["x"], :3]
        assert np.max(np.abs(got - np.array(k["rgb"]))) < 1e-6, (k, got)
    img = cache[(256, 256, 0.0)]
    hits = int(((img[..., 0] < 1.0) & (img[..., 2] < 0.9999999)).sum())
    assert hits == kats["hit_pixels_256_t0"]


PATHS = ["jit", "interpreter", "lanes"]
# csg360_nested's specialised kernel (levelled truth tables, ~300 primitives) takes hiprtc
# a minute or two the first time a process builds it
CSG360 = pytest.param("csg360_nested", marks=pytest.mark.timeout(600))


def _scene(name, path="jit", **kw):
    r = wl.Renderer(name, max_nodes=4096)
    info = scenes.build(name, r, **kw) if name in scenes.SCENES else None
    r.set_tracer(path)
    return r, info


def _union_only(r):
    prog, nrec, nprim = r.program()
    pc = 0
    while pc < nrec:
        op = prog[pc].op
        if op == wl.WO_OP_PRIM:
            pc += 1 + prog[pc].u0
            continue
        if op not in (wl.WO_OP_UNION, wl.WO_OP_BOUND):
            return False
        pc += 1
    return nprim > 0


def _union_of_terms(r, max_lits=2):
    """Restatement of trace_kernels.hip extract_terms: the root is a union of terms, each
    a conjunction of at most max_lits literals (a primitive or its complement), and
    every primitive is in one term -- the lane tracer's term mode."""
    prog, nrec, nprim = r.program()
    st = []
    pc = 0
    while pc < nrec:
        op = prog[pc].op
        if op == wl.WO_OP_PRIM:
            st.append(("conj", [(prog[pc].u1, True)]))
            pc += 1 + prog[pc].u0
            continue
        pc += 1
        if op == wl.WO_OP_BOUND:
            continue
        b, a = st.pop(), st.pop()
        out = ("bad", None)
        terms_of = lambda x: [x[1]] if x[0] == "conj" else x[1]
        if a[0] != "bad" and b[0] != "bad":
            if op == wl.WO_OP_UNION:
                out = ("union", terms_of(a) + terms_of(b))
            elif op == wl.WO_OP_INTER and a[0] == b[0] == "conj":
                out = ("conj", a[1] + b[1])
            elif op in (wl.WO_OP_DIFF, wl.WO_OP_RDIFF):
                keep, sub = (a, b) if op == wl.WO_OP_DIFF else (b, a)
                singles = terms_of(sub)
                if keep[0] == "conj" and all(len(t) == 1 and t[0][1] for t in singles):
                    out = ("conj", keep[1] + [(t[0][0], False) for t in singles])
        st.append(out)
    if len(st) != 1 or st[0][0] == "bad":
        return False
    terms = [st[0][1]] if st[0][0] == "conj" else st[0][1]
    ords = [o for t in terms for o, _ in t]
    return all(1 <= len(t) <= max_lits for t in terms) and len(ords) == len(set(ords))


def _lanes_eligible(r):
    """The lane tracer takes every scene: union-only (a count), a union of small terms
    (term mode), else the general tree (its value kept per lane, kind 7)."""
    return r.program()[2] > 0


def _check_path(r, path, scene=None):
    """The kernel the tracer setting must have selected (renderer_ext.h Wo_Tracer)."""
    nprim = r.program()[2]
    if path == "interpreter":
        want = "interpreter"
    elif path == "lanes" and _lanes_eligible(r):
        want = "lanes"
    else:
        # JIT up to WOLOLO_JIT_MAX_PRIMS (256) primitives, and above for a general tree the
        # levelled truth tables evaluate (csg360_nested's 309); else the lanes (rtiow_cover's
        # 487, csg512_balanced's union of terms)
        hlut = nprim > 256 and "#define WO_JIT_HLUT 1\n" in (r.jit_source() or "")
        want = "jit" if (0 < nprim <= 256 or hlut) else ("lanes" if _lanes_eligible(r) else "interpreter")
    assert r.trace_path() == want, (scene, r.trace_path(), want)


def _oracle_rows(r, params):
    prog, nrec, _ = r.program()
    mats, nm = r.materials()
    fr = r.frame_desc(params)
    img, segs = pyoracle.pathtrace_rows(prog, nrec, mats, nm, fr, 0, params.height)
    return img, segs


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("scene", ["csg32", "csg32_nested", "rtiow_cover", "csg256_balanced", "csg256_chain",
                                   "csg512_balanced", CSG360])
@pytest.mark.parametrize("mode", [wl.MODE_PATHTRACE, wl.MODE_NORMALS])
def test_pathtrace_small_frame_bitexact(scene, mode, path):
    r, info = _scene(scene, path)
    w, h, spp = (48, 27, 4) if scene == "csg360_nested" else (96, 54, 8)  # the oracle's cost: every leaf, every event
    p = info.params(width=w, height=h, spp=spp if mode == wl.MODE_PATHTRACE else 1, mode=mode, seed=7)
    img = r.render(p)
    _check_path(r, path, scene)
    ref, _ = _oracle_rows(r, p)
    _cmp(img, ref, f"{scene} mode={mode} path={path}")
    r.close()


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("scene", ["csg32", "csg32_nested", "rtiow_cover", "csg256_balanced", "csg256_chain",
                                   "csg512_balanced", CSG360])
def test_pathtrace_full_size_sampled_pixels(scene, path):
    """BASELINE configs at full size (1920x1080, 64 spp, 8 bounces): the whole frame on
    the GPU, a random sample of pixels on the oracle.  Every path runs every scene (the
    lane tracer's general form takes the trees that are neither union-only nor a union
    of small terms)."""
    r, info = _scene(scene, path)
    p = info.params()
    img = r.render(p)
    _check_path(r, path, scene)
    assert np.isfinite(img).all()
    rng = np.random.default_rng(1234)
    n = 192
    xs = rng.integers(0, p.width, n).astype(np.uint32)
    ys = rng.integers(0, p.height, n).astype(np.uint32)
    prog, nrec, _ = r.program()
    mats, nm = r.materials()
    ref, _ = pyoracle.pathtrace_pixels(prog, nrec, mats, nm, r.frame_desc(p), xs, ys)
    _cmp(img[ys, xs], ref, f"{scene} full-size sampled")
    r.close()


@pytest.mark.parametrize("path", PATHS)
def test_golden_fixtures_on_gpu(path):
    man = json.load(open(os.path.join(GOLD, "manifest.json")))
    for case in man["pathtrace"]:
        r, info = _scene(case["scene"], path)
        p = info.params(width=case["w"], height=case["h"], spp=case["spp"], mode=case["mode"])
        img = r.render(p)
        ref = np.fromfile(os.path.join(GOLD, case["file"]), dtype=np.float32).reshape(case["h"], case["w"], 4)
        _cmp(img, ref, case["name"])
        r.close()


def test_deterministic_and_seed_sensitive():
    r, info = _scene("csg32")
    p = info.params(width=128, height=72, spp=4)
    a = r.render(p)
    b = r.render(p)
    assert np.array_equal(a, b)
    p2 = info.params(width=128, height=72, spp=4, seed=99)
    c = r.render(p2)
    assert not np.array_equal(a, c)
    r.close()


def test_sample_offset_splits_average():
    """spp linearity: mean of two renders over disjoint sample ranges == one render of
    both ranges (up to fp32 re-association of the per-pixel mean)."""
    r, info = _scene("csg32")
    full = r.render(info.params(width=64, height=36, spp=8))
    h1 = r.render(info.params(width=64, height=36, spp=4, sample_offset=0))
    h2 = r.render(info.params(width=64, height=36, spp=4, sample_offset=4))
    np.testing.assert_allclose((h1 + h2) / 2, full, rtol=0, atol=2e-6)
    r.close()


def _torch():
    import torch
    return torch


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("nranks,tile,band", [(1, 16, (0, 0)), (2, 16, (0, 0)), (3, 8, (0, 0)), (8, 16, (0, 0)),
                                              (5, 7, (0, 0)), (3, 8, (2, 1)), (8, 4, (8, 1)), (4, 4, (3, 2))])
def test_row_tiles_assemble_to_full_frame(nranks, tile, band, path):
    """`band`: weighted row bands (wo_renderer_set_band_weight: rank 0 sits out `skip`
    of every `cycle` rounds), as bench.py gives N-rank frames."""
    torch = _torch()
    r, info = _scene("csg32", path)
    p = info.params(width=200, height=123, spp=2)
    full = r.render(p)
    r.set_band_weight(*band)
    lr = wl.local_rows(p.height, tile, nranks, band)
    gathered = torch.zeros((nranks, lr, p.width, 4), dtype=torch.float32, device="cuda")
    seg = torch.zeros(1, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for rank in range(nranks):
        r.render_rows_device(p, gathered[rank].data_ptr(), tile, rank, nranks, stream, seg.data_ptr())
    frame = torch.empty((p.height, p.width, 4), dtype=torch.float32, device="cuda")
    wl.assemble_rows_device(gathered.data_ptr(), frame.data_ptr(), p.width, p.height, tile, nranks, stream, band)
    torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy(), full)
    # segment counter == oracle's count for the whole frame
    _, segs = _oracle_rows(r, p)
    assert int(seg.item()) == segs
    r.close()


def test_c4_csg32_4k_row_tiles_of_8_ranks():
    """BASELINE config C4 (csg32, 3840x2160, 256 spp, row tiles over 8 GPUs + one gather):
    the 8 ranks' shares rendered one after another on this GPU, each into its slice of
    one rank-major buffer (what the gather delivers to rank 0), then un-interleaved.
    The assembled frame equals one full-frame render bit for bit, 192 sampled pixels
    equal the oracle's, and the 8 shares' segment counts add up to the full frame's."""
    torch = _torch()
    r, info = _scene("csg32", "jit")
    p = info.params(width=3840, height=2160, spp=256)
    T, N = 4, 8
    lr = wl.local_rows(p.height, T, N)
    stream = torch.cuda.current_stream().cuda_stream
    full = torch.empty((p.height, p.width, 4), dtype=torch.float32, device="cuda")
    seg_full = torch.zeros(1, dtype=torch.int64, device="cuda")
    r.render_rows_device(p, full.data_ptr(), T, 0, 1, stream, seg_full.data_ptr())
    gathered = torch.zeros((N, lr, p.width, 4), dtype=torch.float32, device="cuda")
    seg = torch.zeros(N, dtype=torch.int64, device="cuda")
    for rank in range(N):
        r.render_rows_device(p, gathered[rank].data_ptr(), T, rank, N, stream, seg[rank:].data_ptr())
    frame = torch.empty_like(full)
    wl.assemble_rows_device(gathered.data_ptr(), frame.data_ptr(), p.width, p.height, T, N, stream)
    torch.cuda.synchronize()
    assert torch.equal(frame, full), "assembled 8-rank frame differs from the full render"
    assert int(seg.sum().item()) == int(seg_full.item())
    # every rank got a share of the work (row-cyclic tiles balance it within a few %)
    shares = seg.cpu().numpy().astype(np.float64)
    assert shares.min() > 0.9 * shares.mean(), shares
    img = full.cpu().numpy()
    assert np.isfinite(img).all()
    rng = np.random.default_rng(4321)
    n = 192
    xs = rng.integers(0, p.width, n).astype(np.uint32)
    ys = rng.integers(0, p.height, n).astype(np.uint32)
    prog, nrec, _ = r.program()
    mats, nm = r.materials()
    ref, _ = pyoracle.pathtrace_pixels(prog, nrec, mats, nm, r.frame_desc(p), xs, ys)
    _cmp(img[ys, xs], ref, "C4 csg32 4K 256spp sampled")
    r.close()


@pytest.mark.parametrize("path", PATHS)
def test_event_window_overflow_restart(path):
    """A ray crossing > 8 primitive boundaries exercises the window re-collection path."""
    r = wl.Renderer("overflow", max_nodes=256)
    r.set_tracer(path)
    items = []
    for i in range(24):  # a row of overlapping spheres along -z in front of the camera
        s = r.sphere(0.6)
        items.append((s, (0.05 * (i % 3), 0.0, -2.0 - 0.5 * i)))
    # difference chain makes many events non-flipping
    node, off = items[0]
    acc = r.union(wl.arg(node, off), wl.arg(items[1][0], items[1][1]))
    for k, (s, c) in enumerate(items[2:]):
        op = r.difference if k % 2 else r.union
        acc = op(wl.arg(acc), wl.arg(s, c))
    r.set_camera((0, 0, 0), (0, 0, -1), (0, 1, 0), 30.0)
    for mode, spp in [(wl.MODE_NORMALS, 1), (wl.MODE_PATHTRACE, 4)]:
        p = wl.render_params(48, 48, spp=spp, max_depth=6, mode=mode)
        img = r.render(p)
        _check_path(r, path)
        ref, _ = _oracle_rows(r, p)
        _cmp(img, ref, f"overflow mode={mode} path={path}")
    r.close()


@pytest.mark.parametrize("path", PATHS)
def test_edge_scenes(path):
    # empty scene: sky only
    r = wl.Renderer("empty", max_nodes=4)
    r.set_tracer(path)
    p = wl.render_params(32, 16, spp=2, mode=wl.MODE_PATHTRACE)
    img = r.render(p)
    ref, segs = _oracle_rows(r, p)
    _cmp(img, ref, "empty scene")
    assert segs == 32 * 16 * 2
    r.close()
    # a lone ground half-space (unbounded), a zero-radius sphere, a degenerate normal
    r = wl.Renderer("edges", max_nodes=16)
    r.set_tracer(path)
    g = r.halfspace((0, 1, 0))
    z = r.sphere(0.0)
    dgn = r.halfspace((0, 0, 0))
    s = r.sphere(0.5)
    u = r.union(wl.arg(g, (0, -0.5, 0)), wl.arg(z, (0, 0, -1)))
    i = r.intersection(wl.arg(dgn), wl.arg(s, (0.3, 0.0, -1.5)))
    r.union(wl.arg(u), wl.arg(i))
    r.set_material(s, r.dielectric(1.5))
    r.set_camera((0, 0.3, 1), (0, 0, -1), (0, 1, 0), 60.0, 0.05, 2.0)
    for mode, spp in [(wl.MODE_NORMALS, 1), (wl.MODE_PATHTRACE, 4)]:
        p = wl.render_params(64, 48, spp=spp, max_depth=8, mode=mode)
        img = r.render(p)
        _check_path(r, path)
        ref, _ = _oracle_rows(r, p)
        _cmp(img, ref, f"edge scene mode={mode} path={path}")
    r.close()


def _axis_center_dir(fr):
    """The normals-mode ray direction of the centre pixel, as the kernels compute it (fp32)."""
    f32 = np.float32
    c = fr.cam
    x, y = fr.width // 2, fr.height // 2
    sx = f32(f32(x) + f32(0.5)) * f32(fr.inv_width)
    ty = f32(f32(fr.height - 1 - y) + f32(0.5)) * f32(fr.inv_height)
    return [f32(f32(f32(c.lower_left[i]) + sx * f32(c.horizontal[i])) + ty * f32(c.vertical[i])) - f32(c.origin[i])
            for i in range(3)]


@pytest.mark.parametrize("path", ["jit", "interpreter"])
def test_axis_parallel_rays_through_slabs(path):
    """Rays parallel to box faces (a direction component exactly 0): the specialised
    kernel's fused slab-pair path falls back to the per-face form there.  The centre
    pixel looks straight down -z, the centre row has d.y = 0, and a fuzz-free mirror
    face sends rays straight back along +z."""
    r = wl.Renderer("slabs", max_nodes=64)
    r.set_tracer(path)
    front, front_planes = scenes._box_extents(r, (0.0, 0.0, -3.0), (0.5, 0.5, 0.5))
    back, _ = scenes._box_extents(r, (0.0, 0.0, 4.0), (2.0, 2.0, 0.5))
    side, side_planes = scenes._box_extents(r, (1.5, 0.0, -5.0), (0.5, 1.0, 0.5))
    u = r.union(wl.arg(front), wl.arg(back))
    r.union(wl.arg(u), wl.arg(side))
    mirror, clay = r.metal((0.9, 0.9, 0.9), 0.0), r.lambertian((0.2, 0.6, 0.3))
    for pl in front_planes:
        r.set_material(pl, mirror)
    for pl in side_planes:
        r.set_material(pl, clay)
    r.set_camera((0, 0, 0), (0, 0, -1), (0, 1, 0), 60.0, 0.0, 1.0)
    for mode, spp in [(wl.MODE_NORMALS, 1), (wl.MODE_PATHTRACE, 4)]:
        p = wl.render_params(33, 33, spp=spp, max_depth=4, mode=mode, seed=3)
        if mode == wl.MODE_NORMALS:
            dx, dy, dz = _axis_center_dir(r.frame_desc(p))
            assert dx == 0.0 and dy == 0.0 and dz < 0.0, (dx, dy, dz)
        img = r.render(p)
        ref, _ = _oracle_rows(r, p)
        _cmp(img, ref, f"slabs mode={mode} path={path}")
    r.close()


def _union_scene(n_spheres=90):
    """Union-only scene for the lane tracer: overlapping spheres (long event runs, window
    overflow and BOUND pruning barriers), two boxes (6-plane convex primitives), a ground
    half-space, glass spheres (bounces that start inside the solid) and metal."""
    r = wl.Renderer("lanes-union", max_nodes=1024)
    rng = np.random.default_rng(5)
    glass, steel, clay = r.dielectric(1.5), r.metal((0.8, 0.8, 0.9), 0.1), r.lambertian((0.6, 0.4, 0.3))
    items = []
    for i in range(n_spheres):
        s = r.sphere(float(rng.uniform(0.2, 0.7)))
        r.set_material(s, [glass, steel, clay][i % 3])
        items.append(wl.arg(s, tuple(float(v) for v in (rng.uniform(-3, 3), rng.uniform(0, 2), rng.uniform(-8, 0)))))
    for cx in (-1.5, 1.5):
        planes = [r.halfspace(n) for n in ((1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1))]
        acc = wl.arg(planes[0], (0.5, 0, 0))
        for h, n in zip(planes[1:], ((-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1))):
            acc = wl.arg(r.intersection(acc, wl.arg(h, tuple(0.5 * v for v in n))))
        items.append(wl.arg(acc.node, (cx, 0.6, -2.0)))
    ground = r.halfspace((0, 1, 0))
    items.append(wl.arg(ground, (0, -0.2, 0)))
    while len(items) > 1:
        nxt = [wl.arg(r.union(items[i], items[i + 1])) for i in range(0, len(items) - 1, 2)]
        if len(items) % 2:
            nxt.append(items[-1])
        items = nxt
    r.set_camera((0.3, 1.0, 4.0), (0.0, 0.8, -3.0), (0, 1, 0), 50.0)
    return r


@pytest.mark.parametrize("tracer", ["lanes", "auto"])
def test_lanes_union_scene_bitexact(tracer, monkeypatch):
    # AUTO takes the lane tracer for union-only scenes above WOLOLO_LANES_MIN_PRIMS (256 by default)
    monkeypatch.setenv("WOLOLO_LANES_MIN_PRIMS", "64")
    r = _union_scene()
    assert _union_only(r) and r.program()[2] > 64
    r.set_tracer(tracer)
    for mode, spp in [(wl.MODE_NORMALS, 1), (wl.MODE_PATHTRACE, 4)]:
        p = wl.render_params(80, 60, spp=spp, max_depth=8, mode=mode, seed=3)
        img = r.render(p)
        assert r.trace_path() == "lanes"
        ref, _ = _oracle_rows(r, p)
        _cmp(img, ref, f"union scene mode={mode} tracer={tracer}")
    r.close()


def test_lanes_bvh_depth_bound(monkeypatch):
    """A chain of spheres at exponentially growing spacing: binned SAH splits off one
    far sphere at a time, a tree as deep as the scene is long without the depth
    bound.  build_lbvh bounds the depth (log2(n) + 6 levels) so the per-lane LDS
    stack, sized by the depth, never overflows, and the image stays the oracle's."""
    monkeypatch.setenv("WOLOLO_LANES_MIN_PRIMS", "64")
    r = wl.Renderer("deep", max_nodes=4096)
    n = 600
    items = []
    for i in range(n):
        s = r.sphere(0.05 + 0.02 * (i % 3))
        x = 0.1 * (1.02 ** i - 1.0)
        items.append(wl.arg(s, (x - 3.0, 0.3 * np.sin(i), -0.2 * (i % 5))))
    while len(items) > 1:
        nxt = [wl.arg(r.union(items[i], items[i + 1])) for i in range(0, len(items) - 1, 2)]
        if len(items) % 2:
            nxt.append(items[-1])
        items = nxt
    r.set_camera((-3.5, 0.5, 3.0), (0.0, 0.0, -1.0), (0, 1, 0), 60.0)
    r.set_tracer("lanes")
    p = wl.render_params(64, 40, spp=2, max_depth=6, mode=wl.MODE_PATHTRACE, seed=7)
    img = r.render(p)
    assert r.trace_path() == "lanes"
    info = r.lanes_info()
    log2n = int(np.ceil(np.log2(n)))
    assert info["depth"] <= log2n + 6, info
    assert info["nodes"] == n - info["always"] - 1  # a binary tree over the boxed primitives
    ref, _ = _oracle_rows(r, p)
    _cmp(img, ref, "deep chain")
    r.close()


# the lane tracer's form per scene (PathKind: 2 generic primitives, 3 single spheres,
# 6 term mode over <= 256 terms, 14 the resumable 4-wide term-mode walk)
_LANE_KIND = {"union90": 2, "rtiow_cover": 3, "deep600": 3, "glass200": 3, "csg32": 6, "csg256_balanced": 6,
              "csg512_balanced": 14, "csg32_nested": 7, "csg256_chain": 7, "csg360_nested": 7}


@pytest.mark.parametrize("scene", ["union90", "rtiow_cover", "csg32", "csg256_balanced", "deep600", "glass200",
                                   "csg512_balanced", "csg32_nested", "csg256_chain", "csg360_nested"])
def test_lane_tracer_forms_bitexact(scene, monkeypatch):
    """Every form of the lane tracer, each on the scenes that take it: the binary walk
    over generic primitives (boxes, half-spaces: the union scene), over single spheres
    (the RTIOW cover; the 600-sphere chain whose tree is as deep as the depth bound
    allows; a cluster of overlapping glass spheres, rays that start inside), term mode
    over <= 256 terms (csg32, csg256 balanced), the resumable 4-wide term-mode walk
    (csg512_balanced: a wave's walking lanes bail out once few lanes walk, the others
    shade and fetch new rays) and the general tree (csg32_nested, the csg256 chain,
    csg360_nested: events in key order, the tree's value kept per lane); every image
    the oracle's bit for bit."""
    monkeypatch.setenv("WOLOLO_LANES_MIN_PRIMS", "64")
    if scene == "union90":
        r = _union_scene()
        p = wl.render_params(80, 60, spp=4, max_depth=8, mode=wl.MODE_PATHTRACE, seed=3)
    elif scene == "deep600":
        r = wl.Renderer("deep", max_nodes=4096)
        items = []
        for i in range(600):
            s = r.sphere(0.05 + 0.02 * (i % 3))
            items.append(wl.arg(s, (0.1 * (1.02 ** i - 1.0) - 3.0, 0.3 * np.sin(i), -0.2 * (i % 5))))
        while len(items) > 1:
            nxt = [wl.arg(r.union(items[i], items[i + 1])) for i in range(0, len(items) - 1, 2)]
            if len(items) % 2:
                nxt.append(items[-1])
            items = nxt
        r.set_camera((-3.5, 0.5, 3.0), (0.0, 0.0, -1.0), (0, 1, 0), 60.0)
        p = wl.render_params(64, 40, spp=2, max_depth=6, mode=wl.MODE_PATHTRACE, seed=7)
    elif scene == "glass200":
        r = wl.Renderer("glass", max_nodes=1024)
        rng = np.random.default_rng(11)
        glass, clay = r.dielectric(1.5), r.lambertian((0.6, 0.5, 0.4))
        items = []
        for i in range(200):
            sph = r.sphere(float(rng.uniform(0.15, 0.6)))
            r.set_material(sph, glass if i % 2 else clay)
            items.append(wl.arg(sph, tuple(float(v) for v in (rng.uniform(-2, 2), rng.uniform(-1, 1), rng.uniform(-4, 0)))))
        while len(items) > 1:
            nxt = [wl.arg(r.union(items[i], items[i + 1])) for i in range(0, len(items) - 1, 2)]
            if len(items) % 2:
                nxt.append(items[-1])
            items = nxt
        r.set_camera((0.0, 0.0, 3.0), (0.0, 0.0, -2.0), (0, 1, 0), 60.0)
        p = wl.render_params(64, 48, spp=4, max_depth=8, mode=wl.MODE_PATHTRACE, seed=5)
    else:
        r, info = _scene(scene, "lanes")
        p = info.params(width=48, height=27, spp=4, seed=7) if scene == "csg360_nested" else \
            info.params(width=96, height=54, spp=8, seed=7)
    r.set_tracer("lanes")
    for mode in (wl.MODE_NORMALS, wl.MODE_PATHTRACE):
        p.mode = mode
        img = r.render(p)
        assert r.trace_path() == "lanes"
        ref, _ = _oracle_rows(r, p)
        _cmp(img, ref, f"lanes {scene} mode={mode}")
    info = r.lanes_info()
    assert info["kind"] == _LANE_KIND[scene], info
    if info["kind"] == 14:
        assert info["depth"] % 3 == 0 and info["depth"] <= 3 * 24, info  # 3 stack entries per 4-wide level
    r.close()


@pytest.mark.timeout(600)
def test_auto_tracer_choices(monkeypatch):
    """AUTO: the RTIOW cover (union-only, 487 primitives) takes the lane tracer; csg32 and a
    128-primitive union-only scene the JIT; csg512_balanced (427 primitives, a union of
    small terms) the lane tracer's resumable 4-wide term-mode walk; csg360_nested (309
    primitives of a general tree) the JIT with levelled truth tables, or with
    WOLOLO_JIT_GENERAL=0 the lane tracer's general form."""
    for name, want in [("rtiow_cover", "lanes"), ("csg32", "jit"), ("csg256_balanced_union", "jit"),
                       ("csg512_balanced", "lanes"), ("csg360_nested", "jit"), ("csg360_nested", "lanes")]:
        if name == "csg360_nested" and want == "lanes":
            monkeypatch.setenv("WOLOLO_JIT_GENERAL", "0")  # the lanes' general form instead
        r, info = _scene(name, "auto")
        r.render(info.params(width=32, height=18, spp=1))
        if name == "csg360_nested" and want == "jit":
            # a batch render does not wait for the big tree's compile (the lanes meanwhile,
            # test_big_general_tree_renders_on_the_lanes_while_it_compiles); prepare() does
            assert r.trace_path() in ("jit", "lanes"), r.trace_path()
            r.prepare()
            r.render(info.params(width=32, height=18, spp=1))
        assert r.trace_path() == want, (name, r.trace_path())
        if name == "rtiow_cover":
            assert r.lanes_info()["kind"] == 3, r.lanes_info()  # kLanesBvhSpheres: the binary walk
        if name == "csg512_balanced":
            # > 256 terms: the resumable 4-wide walk in term mode (kLanesDynWideTerms)
            assert r.lanes_info()["kind"] == 14, r.lanes_info()
        if name == "csg360_nested" and want == "jit":
            # > 256 primitives of a general tree: the specialised kernel's levelled truth tables
            assert "#define WO_JIT_HLUT 1" in r.jit_source()
        if name == "csg360_nested" and want == "lanes":
            assert r.lanes_info()["kind"] == 7, r.lanes_info()  # kLanesGeneral
        r.close()


@pytest.mark.timeout(600)
def test_big_general_tree_renders_on_the_lanes_while_it_compiles(monkeypatch):
    """a batch render (render_f32) of a general tree above 256 primitives under
    AUTO used to compile its specialised kernel inline (1-2 minutes of hiprtc for
    csg360_nested).  With the code object in neither cache it now starts the compile in
    the background and renders on the lane tracer meanwhile -- the same image bit for
    bit -- and prepare() waits for the kernel and loads it."""
    # a flag no other test uses: the code object is in neither cache
    monkeypatch.setenv("WOLOLO_JIT_FLAGS", f"-DWO_TEST_NONCE={os.getpid()}")
    r, info = _scene("csg360_nested", "auto")
    p = info.params(width=48, height=27, spp=2, seed=3)
    t0 = time.perf_counter()
    img0 = r.render(p)
    dt = time.perf_counter() - t0
    assert r.trace_path() == "lanes" and r.jit_pending(), (r.trace_path(), r.jit_pending())
    img1 = r.render(p)  # another batch render: still no wait while the lanes are loaded
    r.prepare()
    assert not r.jit_pending()
    img2 = r.render(p)
    assert r.trace_path() == "jit", r.trace_path()
    assert np.array_equal(img0, img1) and np.array_equal(img0, img2)
    ref, _ = _oracle_rows(r, p)
    _cmp(img2, ref, "csg360_nested after prepare")
    print(f"first batch render on the lanes: {dt:.2f} s")
    r.close()


def test_kernel_info_names_the_code_object():
    """wo_renderer_kernel_info: the last launch's code object as the runtime loaded it --
    the specialised kernel's key (a SHA-256 of source, options and toolchain: another
    scene, another key), its scratch bytes per lane (csg32's kernel spills nothing) and
    VGPRs; a lane-tracer launch names its template kind, as lanes_info does.  bench.py
    records it in every line and keys the committed traffic figures by it."""
    r, info = _scene("csg32", "auto")
    assert r.kernel_info() is None  # no path launch yet
    r.render(info.params(width=64, height=32, spp=1))
    k = r.kernel_info()
    assert r.trace_path() == "jit" and len(k["key"]) == 64 and int(k["key"], 16) >= 0
    assert k["scratch_bytes"] == 0 and 0 < k["vgprs"] <= 64 and k["lds_bytes"] > 0, k
    # the counting variant (same kernel name, another module) does not change what it reports
    r.count_work(info.params(width=64, height=32, spp=1))
    assert r.kernel_info() == k, (r.kernel_info(), k)
    r2, info2 = _scene("csg32_nested", "auto")
    r2.render(info2.params(width=64, height=32, spp=1))
    k2 = r2.kernel_info()
    assert k2["key"] != k["key"]
    # loaded after csg32's counting variant (a kernel of the same name in another
    # module): its own code object's resources, as its kernel descriptor states them
    import torch

    arch = torch.cuda.get_device_properties(0).gcnArchName
    assert (k2["scratch_bytes"], k2["lds_bytes"]) == wl.jit_code_resources(r2.jit_source(), arch), k2
    r3, info3 = _scene("rtiow_cover", "auto")
    r3.render(info3.params(width=64, height=32, spp=1))
    k3 = r3.kernel_info()
    assert r3.trace_path() == "lanes" and k3["key"].startswith(f"static:{r3.lanes_info()['kind']}:"), k3
    assert len(k3["key"].split(":")[2]) == 40  # the library kernels' source hash
    for x in (r, r2, r3):
        x.close()


@pytest.mark.parametrize("window", ["lds2", "default"])
def test_jit_event_windows(window, monkeypatch):
    """The specialised kernel's event windows -- the sorted LDS list (csg32_nested),
    the register window (csg256_chain) -- and the LDS list's overflow barrier
    (capacity 2 forces it on most rays that meet more than one primitive) all give
    the oracle's frame."""
    if window == "lds2":
        monkeypatch.setenv("WOLOLO_JIT_FLAGS", "-DWO_LDS_EVENTS=2")
    for name in ["csg32", "csg32_nested", "csg256_chain"]:
        r, info = _scene(name, "jit")
        p = info.params(width=64, height=36, spp=4, seed=11)
        img = r.render(p)
        _check_path(r, "jit")
        ref, _ = _oracle_rows(r, p)
        _cmp(img, ref, f"{name} window={window}")
        r.close()


@pytest.mark.parametrize("flags", [
    "-DWO_LDS_NEXT_EAGER=0",
    "-DWO_LDS_NEXT_EAGER=7",
    "-DWO_LDS_EVENTS=2 -DWO_LDS_NEXT_EAGER=7",  # eager reads clamped to the list
    "-DWO_LDS_KEEP_SMALLEST=0",  # a full event list keeps its first keys
    "-DWO_LDS_EVENTS=3",  # ... or its 3 smallest (overflow on most nested rays)
])
def test_jit_compile_flag_variants(flags, monkeypatch):
    """The event list's compile-time variants (WOLOLO_JIT_FLAGS) change how much work a
    wave does, never the image: every setting gives the oracle's frame on the scenes
    with multi-member primitives (csg32's lenses and rounded cube, csg32_nested's
    boxes, csg256 balanced's 21 sphere intersections)."""
    monkeypatch.setenv("WOLOLO_JIT_FLAGS", flags)
    for name in ["csg32", "csg32_nested", "csg256_balanced"]:
        r, info = _scene(name, "jit")
        p = info.params(width=64, height=36, spp=4, seed=13)
        img = r.render(p)
        _check_path(r, "jit")
        ref, _ = _oracle_rows(r, p)
        _cmp(img, ref, f"{name} {flags}")
        r.close()


@pytest.mark.parametrize("tile", ["8x8", "8x4", "4x4"])
@pytest.mark.parametrize("path", PATHS)
def test_workgroup_tile_shapes(tile, path, monkeypatch):
    """Every workgroup tile shape the launch can pick gives the oracle's frame, on
    a frame whose edges cut tiles (odd width, odd height)."""
    monkeypatch.setenv("WOLOLO_TILE", tile)
    r, info = _scene("csg32", path)
    p = info.params(width=77, height=43, spp=3, seed=5)
    img = r.render(p)
    _check_path(r, path, "csg32")
    ref, _ = _oracle_rows(r, p)
    _cmp(img, ref, f"tile {tile} path={path}")
    r.close()


def test_progressive_accumulation_equals_one_render():
    """k accumulated renders of s samples == one render of k*s samples, bit for bit
    (exact fixed-point sums carried across launches), from a non-zero sample offset."""
    r, info = _scene("csg32", "jit")
    base = info.params(width=72, height=40, spp=3, seed=9, sample_offset=5)
    img = None
    for k in range(4):
        img, n = r.render_accumulate(base, reset=(k == 0))
        assert n == 3 * (k + 1)
    full = r.render(info.params(width=72, height=40, spp=12, seed=9, sample_offset=5))
    _cmp(img, full, "progressive 4 x 3 spp vs 12 spp")
    ref, _ = _oracle_rows(r, info.params(width=72, height=40, spp=12, seed=9, sample_offset=5))
    _cmp(img, ref, "progressive vs oracle")
    r.close()


def test_draw_frame_pipeline_and_progressive():
    """draw_frame keeps one frame in flight and presents in order; with progressive
    accumulation the presented frame after k draws is the k*spp render; a camera
    change starts over."""
    r, info = _scene("csg32", "jit")
    p = info.params(width=64, height=36, spp=2, seed=4)
    r.set_draw_params(p)
    # plain pipeline: every frame is the same render
    for _ in range(3):
        r.draw_frame()
    r.finish()
    _cmp(r.last_frame(), r.render(p), "pipelined draw_frame")
    # progressive: 3 draws accumulate 6 samples
    r.set_progressive(True)
    for _ in range(3):
        r.draw_frame()
    r.finish()
    assert r.accumulated_spp() == 6
    _cmp(r.last_frame(), r.render(info.params(width=64, height=36, spp=6, seed=4)), "progressive draw_frame")
    # a camera change restarts the accumulation
    r.set_camera((0.0, 4.0, 10.0), (0.0, 0.6, 0.0), (0, 1, 0), 45.0)
    r.draw_frame()
    r.finish()
    assert r.accumulated_spp() == 2
    _cmp(r.last_frame(), r.render(p), "progressive after a camera change")
    r.close()
