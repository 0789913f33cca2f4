"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_float, c_int, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
_lib = None


def build(quiet: bool = True):
    subprocess.run(["make", "-C", HERE], check=True, stdout=subprocess.DEVNULL if quiet else None)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        lib.oracle_ubershader_pixel.argtypes = [POINTER(c_float), c_uint32, c_uint32, c_uint32, c_uint32, c_float,
                                                c_uint32]
        lib.oracle_ubershader_frame.argtypes = [c_void_p, c_uint32, c_uint32, c_float, c_uint32, c_int]
        lib.oracle_pathtrace_pixels.argtypes = [c_void_p, c_uint32, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p,
                                                c_uint32, c_void_p, POINTER(c_uint64), c_int]
        lib.oracle_pathtrace_pixels.restype = c_int
        lib.oracle_pathtrace_rows.argtypes = [c_void_p, c_uint32, c_void_p, c_uint32, c_void_p, c_uint32, c_uint32,
                                              c_void_p, POINTER(c_uint64), c_int]
        lib.oracle_pathtrace_rows.restype = c_int
        lib.oracle_trace.argtypes = [c_void_p, c_uint32, POINTER(c_float), POINTER(c_float), POINTER(c_float),
                                     POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)]
        lib.oracle_trace.restype = c_int
        lib.oracle_pcg_hash.argtypes = [c_uint32]
        lib.oracle_pcg_hash.restype = c_uint32
        lib.oracle_rng_next.argtypes = [POINTER(c_uint32)]
        lib.oracle_rng_next.restype = c_uint32
        _lib = lib
    return _lib


def host_cpus() -> int:
    """CPUs this process may run on (sched_getaffinity)."""
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        return max(1, os.cpu_count() or 1)


def cpu_quota():
    """The cgroup's CPU bandwidth limit in CPUs (cgroup v2 cpu.max, or v1
    cfs_quota_us / cfs_period_us), rounded up; None when unlimited or unknown."""
    import math
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, math.ceil(int(q) / int(per)))
        return None
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return max(1, math.ceil(q / per)) if q > 0 and per > 0 else None
    except (OSError, ValueError):
        return None


def usable_cpus() -> int:
    """The CPUs this process can use at once: the affinity mask, capped by the
    cgroup's CPU quota (the GPU box: 256 CPUs in the mask, a 16-CPU quota -- more
    threads than the quota only time-share it)."""
    n, q = host_cpus(), cpu_quota()
    return min(n, q) if q else n


def threads_source() -> str:
    n = os.environ.get("OMP_NUM_THREADS")
    if n and n.isdigit() and int(n) != usable_cpus():
        return "OMP_NUM_THREADS override"
    return "affinity mask capped by the cgroup CPU quota" if cpu_quota() else "affinity mask"


def nthreads_default() -> int:
    """Every usable CPU (usable_cpus); OMP_NUM_THREADS only as an explicit override
    that differs from it (threads_source names which applied)."""
    n = os.environ.get("OMP_NUM_THREADS")
    if n and n.isdigit() and int(n) != usable_cpus():
        return max(1, int(n))
    return usable_cpus()


def ubershader_pixel(x, y, w, h, t, mode=0):
    o = (c_float * 4)()
    load().oracle_ubershader_pixel(o, x, y, w, h, float(t), mode)
    return np.array(o[:], dtype=np.float32)


def ubershader_frame(w, h, t, mode=0, nthreads=None) -> np.ndarray:
    out = np.empty((h, w, 4), dtype=np.float32)
    load().oracle_ubershader_frame(out.ctypes.data, w, h, float(t), mode, nthreads or nthreads_default())
    return out


def pathtrace_pixels(prog, n_recs, mats, n_mats, frame, xs, ys, nthreads=None):
    xs = np.ascontiguousarray(xs, dtype=np.uint32)
    ys = np.ascontiguousarray(ys, dtype=np.uint32)
    out = np.empty((len(xs), 4), dtype=np.float32)
    segs = c_uint64(0)
    rc = load().oracle_pathtrace_pixels(ctypes.addressof(prog), n_recs, ctypes.addressof(mats), n_mats,
                                        ctypes.addressof(frame), xs.ctypes.data, ys.ctypes.data, len(xs),
                                        out.ctypes.data, ctypes.byref(segs), nthreads or nthreads_default())
    if rc:
        raise RuntimeError("oracle_pathtrace_pixels failed")
    return out, segs.value


def pathtrace_rows(prog, n_recs, mats, n_mats, frame, row0, nrows, nthreads=None):
    out = np.empty((nrows, frame.width, 4), dtype=np.float32)
    segs = c_uint64(0)
    rc = load().oracle_pathtrace_rows(ctypes.addressof(prog), n_recs, ctypes.addressof(mats), n_mats,
                                      ctypes.addressof(frame), row0, nrows, out.ctypes.data, ctypes.byref(segs),
                                      nthreads or nthreads_default())
    if rc:
        raise RuntimeError("oracle_pathtrace_rows failed")
    return out, segs.value


def trace(prog, n_recs, o, d):
    of = (c_float * 3)(*o)
    df = (c_float * 3)(*d)
    t = c_float(0)
    p, ty, m, ra = c_uint32(0), c_uint32(0), c_uint32(0), c_uint32(0)
    hit = load().oracle_trace(ctypes.addressof(prog), n_recs, of, df, ctypes.byref(t), ctypes.byref(p),
                              ctypes.byref(ty), ctypes.byref(m), ctypes.byref(ra))
    if hit < 0:
        raise RuntimeError("oracle_trace failed")
    return (t.value, p.value, ty.value, m.value, ra.value) if hit else None
