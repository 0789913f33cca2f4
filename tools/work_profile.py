#!/usr/bin/env python3
"""Executed-work counters and per-section wave cycles of one frame (diagnostic).

Renders one frame of a scene with the counting variant of the specialised kernel
built with -DWO_TIME_SECTIONS=1 (shader-clock stamps around the sections of the
path loop) and prints the work per segment and where the waves' cycles went.

    python tools/work_profile.py csg32 [--width 1920 --height 1080 --spp 64]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scenes", nargs="+")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--tracer", default="auto")
    a = ap.parse_args()
    flags = os.environ.get("WOLOLO_JIT_FLAGS", "")
    os.environ["WOLOLO_JIT_FLAGS"] = (flags + " -DWO_TIME_SECTIONS=1").strip()
    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl
    for name in a.scenes:
        r = wl.Renderer("prof", max_nodes=4096)
        info = scenes.build(name, r)
        r.set_tracer(a.tracer)
        p = info.params(width=a.width, height=a.height, spp=a.spp)
        w = r.count_work(p)
        segs = w["segments"]
        cyc = {k: w[k] for k in wl.WORK_KINDS if k.startswith("cyc_")}
        loop = max(cyc["cyc_loop"], 1)
        out = {"scene": name, "path": r.trace_path(), "segments": segs,
               "per_segment": {k: round(w[k] / segs, 4) for k in wl.WORK_KINDS[1:8]},
               "cycle_share": {k: round(v / loop, 4) for k, v in cyc.items() if k != "cyc_loop"},
               "wave_cycles_per_segment": round(loop / segs, 2),
               # lane iterations without a path (the tile's queue drained), and the
               # sweep loop's lane use (lane steps over 64 x wave trips)
               "idle_lane_iterations": round(w["idle_lanes"] / max(segs + w["idle_lanes"], 1), 4),
               "sweep_lane_use": round(w["sweep_steps"] / max(64 * w["sweep_trips"], 1), 4)}
        print(json.dumps(out), flush=True)
        r.close()


if __name__ == "__main__":
    main()
