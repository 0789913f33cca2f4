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
    ap.add_argument("--rtc", action="store_true",
                    help="compile through hiprtc with the runtime's options (trace_kernels.hip jit_options) "
                         "and read the code object's resource notes, instead of hipcc -S")
    a = ap.parse_args()
    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl
    r = wl.Renderer("isa", max_nodes=4096)
    scenes.build(a.scene, r)
    src = open(a.src).read() if a.src else r.jit_source()
    if a.dump:
        open(a.dump, "w").write(src)
    if a.rtc:
        return rtc(src, a.D, a.keep)
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


def rtc(src, defs, keep):
    """hiprtc compile as jit_compile does (same embedded headers and options)."""
    import ctypes
    lib = ctypes.CDLL("/opt/rocm/lib/libhiprtc.so")
    hdrs = [open(os.path.join(ROOT, "csgrenderer_amd/csrc/wo_device_common.h"), "rb").read(),
            open(os.path.join(ROOT, "include/wololo/wo_scene.h"), "rb").read()]
    names = [b"wo_device_common.h", b"wololo/wo_scene.h"]
    prog = ctypes.c_void_p()
    H = ctypes.c_char_p * 2
    rc = lib.hiprtcCreateProgram(ctypes.byref(prog), src.encode(), b"wo_scene_jit.hip", 2, H(*hdrs), H(*names))
    if rc:
        print("hiprtcCreateProgram", rc)
        return 1
    opts = [b"--offload-arch=gfx950", b"-O3", b"-ffp-contract=off", b"-std=c++17", b"-fno-slp-vectorize"]
    opts += [f"-D{x}".encode() for x in defs]
    extra = os.environ.get("WOLOLO_JIT_FLAGS", "")
    opts += [x.encode() for x in extra.split()]
    O = ctypes.c_char_p * len(opts)
    rc = lib.hiprtcCompileProgram(prog, len(opts), O(*opts))
    if rc:
        n = ctypes.c_size_t()
        lib.hiprtcGetProgramLogSize(prog, ctypes.byref(n))
        log = ctypes.create_string_buffer(n.value + 1)
        lib.hiprtcGetProgramLog(prog, log)
        print(log.value.decode()[-3000:])
        return 1
    n = ctypes.c_size_t()
    lib.hiprtcGetCodeSize(prog, ctypes.byref(n))
    code = ctypes.create_string_buffer(n.value)
    lib.hiprtcGetCode(prog, code)
    d = tempfile.mkdtemp()
    co = os.path.join(d, "k.co")
    open(co, "wb").write(code.raw)
    notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    for key in (".name:", ".vgpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
                ".private_segment_fixed_size", ".group_segment_fixed_size"):
        for line in notes.splitlines():
            if line.strip().startswith(key):
                print(line.strip())
    dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True,
                         text=True).stdout
    print("scratch stores:", dis.count("scratch_store"), "loads:", dis.count("scratch_load"))
    if keep:
        open(keep, "w").write(dis)
    shutil.rmtree(d)
    return 0


if __name__ == "__main__":
    sys.exit(main())
