#!/usr/bin/env python3
"""How much wave-uniform work would ray regrouping save?  (analysis only)

Dumps every ray the CPU oracle traces for a few 8x8 pixel tiles of a scene
(tools/stats/ray_dump.c), groups each tile's rays into waves of 64 under several
policies, and counts per wave the spheres for which at least one lane needs the
sqrt (the specialised kernel's wave-uniform skip) -- the dominant per-primitive
cost of the bounce rays.

    python tools/stats/wave_coherence.py csg32 [--tiles 24]
"""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
os.environ.setdefault("WOLOLO_ALLOW_NO_DEVICE", "1")


def spheres_of(prog, nrec):
    out = []
    for i in range(nrec):
        if prog[i].op == 16:  # WO_LEAF_SPHERE
            out.append([prog[i].f[0], prog[i].f[1], prog[i].f[2], prog[i].f[3]])
    return np.array(out, np.float32)


def need_matrix(rays, sph):
    o = rays[:, None, 0:3]
    d = rays[:, None, 3:6]
    f = o - sph[None, :, 0:3]
    b = (f * d).sum(-1)
    l_ = f - b[..., None] * d
    disc = sph[None, :, 3] - (l_ * l_).sum(-1)
    return (disc >= 0) & ~((b > 0) & (disc < 0.99998 * b * b))


def wave_cost(need, groups):
    """mean over waves of the number of spheres with any needing lane"""
    tot, nw = 0, 0
    for g in groups:
        for k in range(0, len(g), 64):
            idx = g[k:k + 64]
            tot += need[idx].any(axis=0).sum()
            nw += 1
    return tot / max(nw, 1), nw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scene")
    ap.add_argument("--tiles", type=int, default=24)
    ap.add_argument("--spp", type=int, default=64)
    a = ap.parse_args()
    so = "/tmp/wo_ray_dump.so"
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-mfma", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "oracle"), "-o", so, os.path.join(HERE, "ray_dump.c"), "-lm"], check=True)
    lib = ctypes.CDLL(so)
    lib.dump_count.restype = ctypes.c_uint64
    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl
    r = wl.Renderer("wc", max_nodes=8192)
    info = scenes.build(a.scene, r)
    prog, nrec, _ = r.program()
    mats, nm = r.materials()
    params = info.params(spp=a.spp)
    fr = r.frame_desc(params)
    sph = spheres_of(prog, nrec)
    rng = np.random.default_rng(7)
    cap = 64 * a.spp * 40
    buf = np.zeros((cap, 8), np.float32)
    res = {}
    for _ in range(a.tiles):
        tx, ty = int(rng.integers(0, 1920 // 8)), int(rng.integers(0, 1080 // 8))
        xs = np.repeat(np.arange(tx * 8, tx * 8 + 8, dtype=np.uint32)[None], 8, 0).ravel()
        ys = np.repeat(np.arange(ty * 8, ty * 8 + 8, dtype=np.uint32), 8)
        lib.dump_set(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(cap))
        out = np.zeros((64, 4), np.float32)
        segs = ctypes.c_uint64(0)
        lib.oracle_pathtrace_pixels(prog, nrec, mats, nm, ctypes.byref(fr), xs.ctypes.data_as(ctypes.c_void_p),
                                    ys.ctypes.data_as(ctypes.c_void_p), 64, out.ctypes.data_as(ctypes.c_void_p),
                                    ctypes.byref(segs), 1)
        n = min(int(lib.dump_count()), cap)
        rays = buf[:n].copy()
        need = need_matrix(rays, sph)
        depth = rays[:, 6]
        octant = (rays[:, 3] > 0) * 1 + (rays[:, 4] > 0) * 2 + (rays[:, 5] > 0) * 4
        # direction bins: 26 (sign of each component with a dead zone) ~ cube faces/edges/corners
        q = np.sign(np.where(np.abs(rays[:, 3:6]) < 0.4, 0, rays[:, 3:6])).astype(int) + 1
        dbin = q[:, 0] * 9 + q[:, 1] * 3 + q[:, 2]
        prim = depth == 0
        perm = rng.permutation(n)
        pol = {
            "mixed (random within tile)": [perm],
            "primary/secondary split": [np.where(prim)[0], rng.permutation(np.where(~prim)[0])],
            "split + octant sort": [np.where(prim)[0],
                                    np.where(~prim)[0][np.argsort(octant[~prim], kind="stable")]],
            "split + 27-bin direction sort": [np.where(prim)[0],
                                              np.where(~prim)[0][np.argsort(dbin[~prim], kind="stable")]],
        }
        for k, groups in pol.items():
            c, nw = wave_cost(need, groups)
            res.setdefault(k, []).append((c, nw))
        res.setdefault("_rays", []).append((n, int(prim.sum())))
    nr = sum(x[0] for x in res["_rays"])
    npr = sum(x[1] for x in res["_rays"])
    print(f"{a.scene}: {len(sph)} spheres, {nr} rays ({npr} primary) over {a.tiles} tiles of 8x8 x {a.spp} spp")
    for k, v in res.items():
        if k.startswith("_"):
            continue
        tot = sum(c * nw for c, nw in v)
        nw = sum(nw for _, nw in v)
        print(f"  {k:32s} spheres needing sqrt per wave {tot / nw:6.2f}  (waves {nw})")


if __name__ == "__main__":
    main()
