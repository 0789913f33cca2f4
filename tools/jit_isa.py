#!/usr/bin/env python3
"""Compile a scene's generated (specialised) kernel offline with hipcc and report
register use / occupancy / instruction histogram -- for tuning WO_WINDOW and
WO_JIT_MIN_WAVES without a GPU.

    python tools/jit_isa.py csg32 [-D WO_WINDOW=2 -D WO_JIT_MIN_WAVES=4] [--hist]
"""
import argparse
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("WOLOLO_ALLOW_NO_DEVICE", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scene")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--hist", action="store_true")
    ap.add_argument("--keep", default=None, help="copy the .s here")
    ap.add_argument("--src", default=None, help="compile this (edited) generated source instead of the scene's")
    ap.add_argument("--dump", default=None, help="write the scene's generated source here")
    a = ap.parse_args()
    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl
    r = wl.Renderer("isa", max_nodes=4096)
    scenes.build(a.scene, r)
    src = open(a.src).read() if a.src else r.jit_source()
    if a.dump:
        open(a.dump, "w").write(src)
    d = tempfile.mkdtemp()
    os.makedirs(os.path.join(d, "wololo"))
    shutil.copy(os.path.join(ROOT, "csgrenderer_amd/csrc/wo_device_common.h"), d)
    shutil.copy(os.path.join(ROOT, "include/wololo/wo_scene.h"), os.path.join(d, "wololo"))
    open(os.path.join(d, "k.hip"), "w").write("#include <hip/hip_runtime.h>\n" + src)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-I", d, "-c",
           os.path.join(d, "k.hip"), "--cuda-device-only", "-S", "-o", os.path.join(d, "k.s"),
           "-Rpass-analysis=kernel-resource-usage"] + [f"-D{x}" for x in a.D]
    res = subprocess.run(cmd, capture_output=True, text=True)
    for line in res.stderr.splitlines():
        m = re.search(r"remark:\s+(VGPRs|TotalSGPRs|ScratchSize.*|Occupancy.*|SGPRs Spill|VGPRs Spill|LDS Size.*):\s*(\d+)", line)
        if m:
            print(f"{m.group(1)}: {m.group(2)}")
    if res.returncode:
        print(res.stderr[-3000:])
        return 1
    lines = [l.strip() for l in open(os.path.join(d, "k.s")) if l.strip() and not l.strip().startswith((".", ";"))
             and not l.strip().endswith(":")]
    print("instructions:", len(lines))
    if a.hist:
        ops = {}
        for l in lines:
            ops[l.split()[0]] = ops.get(l.split()[0], 0) + 1
        for k, v in sorted(ops.items(), key=lambda x: -x[1])[:30]:
            print(f"  {k:28s}{v}")
    if a.keep:
        shutil.copy(os.path.join(d, "k.s"), a.keep)
    shutil.rmtree(d)
    return 0


if __name__ == "__main__":
    sys.exit(main())
