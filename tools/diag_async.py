#!/usr/bin/env python3
"""Diagnostic: does a hiprtc compile on a host thread block HIP calls of another
thread?  Times small renders while wo_jit_code_object compiles a large scene's
kernel on a Python thread (ctypes drops the GIL during the call)."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (the bench's runtime)
    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl
    os.environ["WOLOLO_JIT_CACHE"] = "0"
    r = wl.Renderer("diag", max_nodes=4096)
    info = scenes.build("csg32", r)
    p = info.params(width=96, height=54, spp=2)
    r.render(p)
    big = wl.Renderer("big", max_nodes=4096)
    scenes.build("csg256_balanced", big)
    src = big.jit_source() + f"\n// {time.time()}\n"
    done = []

    def compile_it():
        t0 = time.perf_counter()
        wl.jit_code_object(src, "gfx950")
        done.append(time.perf_counter() - t0)

    th = threading.Thread(target=compile_it)
    t0 = time.perf_counter()
    th.start()
    times = []
    while not done and time.perf_counter() - t0 < 30:
        a = time.perf_counter()
        r.render(p)
        times.append(time.perf_counter() - a)
    th.join()
    print(f"compile {done[0]:.2f} s on a thread; {len(times)} renders meanwhile, max {max(times) * 1e3:.1f} ms, "
          f"median {sorted(times)[len(times) // 2] * 1e3:.2f} ms")
    t1 = time.perf_counter()
    for _ in range(20):
        r.render(p)
    print(f"renders without a compile: {(time.perf_counter() - t1) / 20 * 1e3:.2f} ms each")


if __name__ == "__main__":
    main()
