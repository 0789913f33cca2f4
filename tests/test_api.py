"""The C-ABI boundary (CPU only): exported symbols, node-store semantics of the
reference (renderer.c:2220-2313), and the reference demo linking unchanged."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from csgrenderer_amd import wololo as wl

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "csgrenderer_amd", "lib")
REF_MAIN = "/root/reference/src/wololo_demo/main.c"


def _declared_functions():
    names = set()
    for dp, _, files in os.walk(INC):
        for f in files:
            if not f.endswith(".h"):
                continue
            src = open(os.path.join(dp, f)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            for m in re.finditer(r"^(?!\s*static)(?!\s*typedef)[A-Za-z_][\w \*]*?\b(wo_\w+)\s*\(", src, flags=re.M):
                names.add(m.group(1))
    return names


def _exported():
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(LIBDIR, "libwololo.so")], check=True,
                         capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_every_declared_symbol_is_exported():
    declared = _declared_functions()
    assert len(declared) >= 30
    exported = _exported()
    missing = sorted(declared - exported)
    assert not missing, f"declared in include/ but not exported: {missing}"


def test_python_mirror_covers_the_abi():
    assert set(wl.SIGNATURES) == _declared_functions()
    wl.load()  # sets every argtype / restype


def test_abi_sizes():
    # renderer.h:22-27 (the reference's by-value operand): sizes measured by SURVEY.md 8(b)
    assert ctypes.sizeof(wl.Vec3) == 24
    assert ctypes.sizeof(wl.Quaternion) == 32
    assert ctypes.sizeof(wl.NodeArgument) == 64


# C type name -> its ctypes mirror in csgrenderer_amd/wololo.py
ABI_MIRRORS = {"Wo_Vec3": wl.Vec3, "Wo_Quaternion": wl.Quaternion, "Wo_Node_Argument": wl.NodeArgument,
               "Wo_RenderParams": wl.RenderParams, "WoRec": wl.WoRec, "WoMaterial": wl.WoMaterial,
               "WoCamera": wl.WoCamera, "WoFrame": wl.WoFrame}


@pytest.mark.parametrize("cname", sorted(ABI_MIRRORS))
def test_abi_mirror_matches_the_c_layout(cname):
    """Every field offset and the size of each ctypes mirror equal what the C compiler laid
    out (wo_abi_layout): a shifted field would corrupt every call that passes the struct."""
    mirror = ABI_MIRRORS[cname]
    assert wl.abi_layout(cname) == ctypes.sizeof(mirror), cname
    for fname, _ in mirror._fields_:
        if fname == "pad":
            continue
        assert wl.abi_layout(cname, fname) == getattr(mirror, fname).offset, (cname, fname)
    assert wl.abi_layout(cname, "no_such_field") == -1
    assert wl.abi_layout("NoSuchType") == -1


def _srgb_ref(v):
    """IEC 61966-2-1 encode in float64 and round-half-up to 8 bits (clamped; NaN -> 0)."""
    v = np.asarray(v, dtype=np.float64)
    c = np.clip(np.nan_to_num(v, nan=0.0), 0.0, 1.0)
    s = np.where(c <= 0.0031308, 12.92 * c, 1.055 * np.power(c, 1.0 / 2.4) - 0.055)
    return np.floor(255.0 * s + 0.5).astype(np.int64), 255.0 * s


def srgb_test_values():
    """Edge values plus a dense sweep of [0, 1] and values either side of every threshold."""
    t = wl.srgb8_thresholds().astype(np.float32)
    around = np.concatenate([t, np.nextafter(t, np.float32(-1)), np.nextafter(t, np.float32(2))])
    edge = np.array([0.0, -0.0, -1.0, 1.0, 2.0, np.inf, -np.inf, np.nan, 1e-45, 0.0031308, 0.04045, 0.5,
                     np.nextafter(np.float32(1), np.float32(0))], dtype=np.float32)
    sweep = np.linspace(0.0, 1.0, 200001, dtype=np.float32)
    return np.concatenate([edge, around.astype(np.float32), sweep])


def test_srgb8_thresholds_and_host_encode():
    """The present encode (renderer.c:813-832 prefers a B8G8R8A8_SRGB swapchain): the table is
    strictly increasing in (0, 1) and the host encode equals the float64 IEC formula for every
    tested value except exact ties (none expected)."""
    t = wl.srgb8_thresholds()
    assert t.shape == (255,) and np.all(np.diff(t) > 0) and t[0] > 0 and t[-1] < 1
    v = srgb_test_values()
    want, x = _srgb_ref(v)
    tie = np.abs(x - np.floor(x) - 0.5) < 1e-9
    rgba = np.stack([v, np.roll(v, 1), np.roll(v, 2), np.ones_like(v)], axis=-1)
    got = wl.srgb8_encode_host(rgba)
    r, g, b, a = (got >> 16) & 255, (got >> 8) & 255, got & 255, got >> 24
    ok = ~tie
    assert np.array_equal(r[ok], want[ok])
    assert np.array_equal(g, np.roll(r, 1)) and np.array_equal(b, np.roll(r, 2))
    assert np.all(a == 255)


def test_node_store_semantics(hostonly):
    """main.c:38-50 prints isroot 0, 0, 1 for two spheres and their union."""
    r = wl.Renderer("Test1Render", max_nodes=8)
    s1 = r.sphere(1.0)
    s2 = r.sphere(1.0)
    blob = r.union(wl.arg(s1), wl.arg(s2))
    assert (s1, s2, blob) == (0, 1, 2)  # sequential handles (renderer.c:2224)
    assert (r.isroot(s1), r.isroot(s2), r.isroot(blob)) == (False, False, True)
    assert r.lib.wo_renderer_node_count(r.ptr) == 3
    assert r.lib.wo_renderer_name(r.ptr) == b"Test1Render"
    assert r.lib.wo_renderer_device(r.ptr) == -1
    r.close()


def test_capacity_and_bad_operands(hostonly):
    r = wl.Renderer("cap", max_nodes=2)
    a = r.sphere(1.0)
    b = r.halfspace((0, 1, 0))
    with pytest.raises(wl.WololoError):
        r.sphere(2.0)  # store full -> WO_NODE_INVALID, no abort
    assert r.lib.wo_renderer_add_union_of_node(r.ptr, wl.arg(a), wl.arg(7)) == wl.WO_NODE_INVALID
    assert r.isroot(a) and r.isroot(b)
    r.close()


def test_empty_name_is_null(hostonly):
    r = wl.Renderer("", max_nodes=1)
    assert r.lib.wo_renderer_name(r.ptr) is None
    r.close()


def test_render_without_device_fails_loudly(hostonly):
    r = wl.Renderer("nodev", max_nodes=4)
    with pytest.raises(wl.WololoError, match="device"):
        r.render(wl.render_params(8, 8))
    r.close()


def test_materials_and_camera(hostonly):
    r = wl.Renderer("mats", max_nodes=4)
    s = r.sphere(1.0)
    m1 = r.lambertian((0.1, 0.2, 0.3))
    m2 = r.metal((0.9, 0.9, 0.9), 2.0)  # fuzz clamps to 1
    m3 = r.dielectric(1.5)
    assert (m1, m2, m3) == (1, 2, 3)
    r.set_material(s, m3)
    u = r.union(wl.arg(s), wl.arg(s, (2, 0, 0)))
    with pytest.raises(wl.WololoError):
        r.set_material(u, m1)  # binops take no material
    mats, n = r.materials()
    assert n == 4 and mats[2].fuzz == 1.0 and mats[3].kind == wl.WO_MAT_DIELECTRIC
    r.set_camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, 0.1, 10.0)
    fr = r.frame_desc(wl.render_params(1920, 1080, spp=64, mode=wl.MODE_PATHTRACE))
    assert fr.cam.lens_radius == pytest.approx(0.05)
    assert list(fr.cam.origin) == [13.0, 2.0, 3.0]
    assert fr.n_prims == 2
    r.close()


@pytest.mark.skipif(not os.path.exists(REF_MAIN), reason="reference demo not present (GPU box)")
def test_reference_demo_links_unchanged(tmp_path):
    """src/wololo_demo/main.c compiles and links, unmodified, against include/ and
    libwololo.so, and prints the reference's isroot answers."""
    exe = tmp_path / "wololo_demo"
    subprocess.run(["gcc", "-std=gnu11", "-O1", "-Wall", "-I", INC, REF_MAIN, "-L", LIBDIR, "-lwololo",
                    f"-Wl,-rpath,{LIBDIR}", "-lm", "-o", str(exe)], check=True)
    env = dict(os.environ, WOLOLO_ALLOW_NO_DEVICE="1", WOLOLO_FRAMES="2")
    res = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=60)
    assert res.returncode == 0, res.stderr
    assert "Sphere1 is root: 0\nSphere2 is root: 0\nBlob is root: 1" in res.stdout
    assert "Quitting..." in res.stdout
