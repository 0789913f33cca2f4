#!/usr/bin/env python3
"""Event statistics of a benchmark scene from the oracle's sweep (analysis only).

    python tools/stats/trace_stats.py csg32 [--rows 32]
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
sys.path.insert(0, os.path.join(ROOT, "oracle"))
os.environ.setdefault("WOLOLO_ALLOW_NO_DEVICE", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scene")
    ap.add_argument("--rows", type=int, default=24)
    ap.add_argument("--spp", type=int, default=8)
    a = ap.parse_args()
    so = "/tmp/wo_trace_stats.so"
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-fopenmp", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "oracle"), "-o", so, os.path.join(HERE, "trace_stats.c"), "-lm"], check=True)
    lib = ctypes.CDLL(so)
    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl
    r = wl.Renderer("st", max_nodes=8192)
    info = scenes.build(a.scene, r)
    prog, nrec, nprim = r.program()
    mats, nm = r.materials()
    params = info.params(width=1920, height=1080, spp=a.spp)
    fr = r.frame_desc(params)
    H = 1080
    rows = np.linspace(0, H - 1, a.rows).astype(np.uint32)
    xs = np.tile(np.arange(1920, dtype=np.uint32), len(rows))
    ys = np.repeat(rows, 1920).astype(np.uint32)
    out = np.zeros((len(xs), 4), np.float32)
    segs = ctypes.c_uint64(0)
    lib.stats_reset()
    lib.oracle_pathtrace_pixels(prog, nrec, mats, nm, ctypes.byref(fr), xs.ctypes.data_as(ctypes.c_void_p),
                                ys.ctypes.data_as(ctypes.c_void_p), len(xs), out.ctypes.data_as(ctypes.c_void_p),
                                ctypes.byref(segs), 8)
    st = (ctypes.c_uint64 * 32)()
    lib.stats_get(st)
    n = st[0]
    print(f"{a.scene}: {nprim} prims, {n} traces, hit {st[1] / n:.3f}, events/trace {st[2] / n:.2f}, "
          f"swept/trace {st[3] / n:.2f}")
    print("swept histogram 0,1,2,3-4,5-8,9+:", " ".join(f"{st[4 + i] / n:.3f}" for i in range(6)))
    print(f"window-4 re-collect {st[10] / n:.4f}, more than 4 events {st[11] / n:.4f}")
    ns, npri = st[16], n - st[16]
    if ns:
        print(f"primary: {npri} traces, hit {(st[1] - st[17]) / npri:.3f}, events {(st[2] - st[18]) / npri:.2f}, "
              f"swept {(st[3] - st[19]) / npri:.2f}")
        print(f"secondary: {ns} traces, hit {st[17] / ns:.3f}, events {st[18] / ns:.2f}, swept {st[19] / ns:.2f}")


if __name__ == "__main__":
    main()
