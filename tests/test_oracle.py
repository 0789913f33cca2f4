"""The CPU oracle against the survey's known answers and the committed fixtures
(CPU only).  This is what pins the oracle before it is trusted as the checker."""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

import pyoracle
from csgrenderer_amd import scenes
from csgrenderer_amd import wololo as wl

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_ubershader_survey_kats():
    kats = json.load(open(os.path.join(GOLD, "ubershader_kats.json")))
    for k in kats["pixels"]:
        got = pyoracle.ubershader_pixel(k["x"], k["y"], k["w"], k["h"], k["t"])
        assert np.max(np.abs(got[:3] - np.array(k["rgb"]))) < 1e-6, k
        assert got[3] == 1.0


def test_ubershader_hit_count_256():
    img = pyoracle.ubershader_frame(256, 256, 0.0)
    hits = int(((img[..., 0] < 1.0) & (img[..., 2] < 0.9999999)).sum())
    assert hits == json.load(open(os.path.join(GOLD, "ubershader_kats.json")))["hit_pixels_256_t0"]


def test_ubershader_properties():
    """Properties of ubershader1.frag that hold at any size: the sky gradient exceeds 1
    below the horizon (frag:116-122 is unclamped), blue is 1 in the sky, the sphere is
    mirror-symmetric in x at time 0."""
    img = pyoracle.ubershader_frame(200, 150, 0.0)
    assert img[-1, 0, 0] > 1.0
    sky = img[0]
    assert np.all(sky[:, 2] == 1.0)
    np.testing.assert_array_equal(img[..., 3], 1.0)
    # the ray direction x is (-a/2 + st.x*a): symmetric about the centre column
    c = img[75, 95:105, 1]
    np.testing.assert_allclose(c, c[::-1], atol=1e-6)


def test_debug_view_is_st():
    img = pyoracle.ubershader_frame(8, 4, 0.0, wl.MODE_DEBUG_ST)
    x = (np.arange(8, dtype=np.float32) + 0.5) / 8
    y = 1.0 - (np.arange(4, dtype=np.float32) + 0.5) / 4
    np.testing.assert_array_equal(img[0, :, 0], x)
    np.testing.assert_array_equal(img[:, 0, 1], y)


def test_sphere_moves_with_time():
    """frag:103: the sphere's centre height is 2 sin(omega t); at t=1 (omega*1 ~ pi/2) it
    sits near y=2, i.e. above the image centre."""
    a = pyoracle.ubershader_frame(192, 108, 0.0)
    b = pyoracle.ubershader_frame(192, 108, 1.0)
    hit_a = np.argwhere(a[..., 2] < 0.9999)
    hit_b = np.argwhere(b[..., 2] < 0.9999)
    assert len(hit_a) and len(hit_b)
    assert hit_b[:, 0].mean() < hit_a[:, 0].mean() - 5


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


def test_ubershader_fixtures():
    man = json.load(open(os.path.join(GOLD, "manifest.json")))
    for c in man["ubershader"]:
        img = pyoracle.ubershader_frame(c["w"], c["h"], c["t"], c["mode"], nthreads=2)
        assert _sha(img) == c["sha256"], c
        if c["file"]:
            ref = np.fromfile(os.path.join(GOLD, c["file"]), dtype=np.float32).reshape(c["h"], c["w"], 4)
            assert np.array_equal(img, ref)


def test_pathtrace_fixtures(hostonly):
    man = json.load(open(os.path.join(GOLD, "manifest.json")))
    for c in man["pathtrace"]:
        r = wl.Renderer(c["name"], max_nodes=4096)
        info = scenes.build(c["scene"], r)
        prog, nrec, _ = r.program()
        assert hashlib.sha256(bytes(prog)[:32 * nrec]).hexdigest() == c["program_sha256"], \
            f"{c['scene']}: scene compiler output changed"
        mats, nm = r.materials()
        p = info.params(width=c["w"], height=c["h"], spp=c["spp"], mode=c["mode"])
        img, segs = pyoracle.pathtrace_rows(prog, nrec, mats, nm, r.frame_desc(p), 0, c["h"], nthreads=4)
        assert segs == c["segments"]
        assert _sha(img) == c["sha256"], c["name"]
        r.close()


# ---- RNG: the oracle's PCG hash vs an independent pure-Python statement ----

def _py_pcg_hash(v):
    s = (v * 747796405 + 2891336453) & 0xFFFFFFFF
    w = (((s >> ((s >> 28) + 4)) ^ s) * 277803737) & 0xFFFFFFFF
    return ((w >> 22) ^ w) & 0xFFFFFFFF


@pytest.mark.parametrize("v", [0, 1, 2, 0xDEADBEEF, 0xFFFFFFFF, 123456789])
def test_pcg_hash_matches_python(v):
    assert pyoracle.load().oracle_pcg_hash(v) == _py_pcg_hash(v)


def test_rng_uniform_in_unit_interval():
    import ctypes
    st = ctypes.c_uint32(12345)
    lib = pyoracle.load()
    vals = [(lib.oracle_rng_next(ctypes.byref(st)) >> 8) * 2.0 ** -24 for _ in range(20000)]
    assert 0.0 <= min(vals) and max(vals) < 1.0
    assert abs(np.mean(vals) - 0.5) < 0.01


def test_sincos_turn_accuracy():
    """The polynomial sin/cos of 2*pi*u used for direction sampling (both kernels and
    oracle): within a few fp32 ulps of float64 sin/cos over [0, 1)."""
    import ctypes
    lib = pyoracle.load()
    lib.oracle_sincos_turn.argtypes = [ctypes.c_float, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    s, c = ctypes.c_float(), ctypes.c_float()
    us = np.concatenate([np.linspace(0, 1, 4001, endpoint=False), np.random.default_rng(0).random(4000)])
    err = 0.0
    for u in us.astype(np.float32):
        lib.oracle_sincos_turn(float(u), ctypes.byref(s), ctypes.byref(c))
        a = 2 * np.pi * float(u)
        err = max(err, abs(s.value - np.sin(a)), abs(c.value - np.cos(a)))
        assert abs(s.value * s.value + c.value * c.value - 1.0) < 1e-6
    assert err < 4e-7, err


def test_sqrt_clamp_is_ieee_sqrt_in_range():
    """The path tracer's sqrt is sqrtf(max(x, 2^-96)). On every input at or
    above 2^-96 it must be IEEE sqrtf bit for bit (numpy's float32 sqrt is correctly
    rounded); only the degenerate inputs below (tiny, zero, negative) deviate from GLSL's
    sqrt, which would give 0 or NaN there. Pins the oracle to IEEE, not to the kernel."""
    import ctypes
    lib = pyoracle.load()
    fp = ctypes.POINTER(ctypes.c_float)
    lib.oracle_sqrt_pt_array.argtypes = [fp, fp, ctypes.c_uint32]
    rng = np.random.default_rng(7)
    lo = np.float32(2.0 ** -96).view(np.uint32)
    hi = np.float32(np.inf).view(np.uint32)
    bits = np.concatenate([rng.integers(lo, hi, 400_000, dtype=np.uint32),
                           np.arange(lo, lo + 4096, dtype=np.uint32),
                           np.array([np.float32(1.0).view(np.uint32), hi - 1, hi], dtype=np.uint32)])
    x = bits.view(np.float32)
    out = np.empty_like(x)
    lib.oracle_sqrt_pt_array(x.ctypes.data_as(fp), out.ctypes.data_as(fp), x.size)
    assert np.array_equal(out.view(np.uint32), np.sqrt(x).view(np.uint32))
    # below the clamp: the documented deviation (finite, = 2^-48) instead of 0 / NaN
    low = np.array([0.0, -0.0, -1.0, 2.0 ** -100, -np.inf], dtype=np.float32)
    out = np.empty_like(low)
    lib.oracle_sqrt_pt_array(low.ctypes.data_as(fp), out.ctypes.data_as(fp), low.size)
    assert np.all(out == np.float32(2.0 ** -48))
