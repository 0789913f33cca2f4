#!/usr/bin/env python3
"""The specialised kernel as compiled by the JIT stack the process loaded: run with
--torch, torch is imported first and its bundled HIP runtime / hiprtc / comgr serve the
library (what bench.py does); without it, the system ROCm's.  Times draw_frame's render
(GPU stamps, median of the last frames) and prints the kernel key and resources.

    python tools/toolchain_ab.py [--torch] csg32 csg32_nested ...
"""
import os
import sys

if "--torch" in sys.argv:
    import torch  # noqa: F401  (its HIP libraries load first)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from csgrenderer_amd import scenes  # noqa: E402
from csgrenderer_amd import wololo as wl  # noqa: E402

stack = sorted({x.split()[-1].split("/")[-1] for x in open("/proc/self/maps") if "hiprtc" in x or "comgr" in x})
for name in [a for a in sys.argv[1:] if not a.startswith("--")]:
    r = wl.Renderer(name, max_nodes=8192)
    info = scenes.build(name, r)
    p = info.params()
    r.set_tracer("auto")
    r.render(p)
    r.prepare()
    r.set_draw_params(p)
    r.set_frame_stamps(True)
    for _ in range(40):
        r.draw_frame()
    r.finish()
    st = r.frame_stamps()[-30:]
    ms = sorted(e - b for b, e, _ in st)
    ki = r.kernel_info()
    print(f"{'torch' if '--torch' in sys.argv else 'system'} {name} render median {ms[len(ms) // 2]:.4f} ms "
          f"min {ms[0]:.4f} ({r.trace_path()}) key {ki['key'][:16]} scratch {ki['scratch_bytes']} vgprs {ki['vgprs']} "
          f"[{' '.join(stack)}]", flush=True)
    r.close()
