"""ctypes mirror of the wololo C API (libwololo.so).

The product is the C-ABI library built from ``csgrenderer_amd/csrc`` (HIP
kernels for gfx950 + C host).  This module only binds it -- same names and
argument meaning as the reference's ``src/wololo/renderer/renderer.h:18-33``
and ``src/wololo/app.h:20-30`` plus the extensions of
``include/wololo/renderer/renderer_ext.h`` -- so tests and ``bench.py`` read
like C callers.  There is no fallback: if the library is missing, loading
raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_bool, c_char_p, c_double, c_float, c_int, c_size_t, c_uint32,
                    c_ulonglong, c_void_p)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# WOLOLO_LIB: another build of the same library (A/B measurements of build options)
LIB_PATH = os.environ.get("WOLOLO_LIB") or os.path.join(PKG_DIR, "lib", "libwololo.so")

# ---- wo_scene.h constants -------------------------------------------------------------------
WO_OP_PRIM, WO_OP_UNION, WO_OP_INTER, WO_OP_DIFF, WO_OP_RDIFF, WO_OP_BOUND = 1, 2, 3, 4, 5, 6
WO_LEAF_SPHERE, WO_LEAF_HALFSPACE = 16, 17
WO_MAT_LAMBERTIAN, WO_MAT_METAL, WO_MAT_DIELECTRIC = 0, 1, 2
MODE_UBERSHADER_RT1, MODE_DEBUG_ST, MODE_PATHTRACE, MODE_NORMALS = 0, 1, 2, 3
TRACER_AUTO, TRACER_INTERPRETER, TRACER_JIT, TRACER_LANES = 0, 1, 2, 3
TRACERS = {"auto": TRACER_AUTO, "interpreter": TRACER_INTERPRETER, "jit": TRACER_JIT, "lanes": TRACER_LANES}
WO_T_MIN = 1.0e-3
# wo_scene.h WO_WORK_* (executed-work counters)
WORK_KINDS = ("segments", "sphere_tests", "halfspace_tests", "bound_tests", "events", "sweep_steps", "recollects",
              "primary_segments", "cyc_take", "cyc_collect", "cyc_sweep", "cyc_shade", "cyc_loop", "idle_lanes",
              "sweep_trips", "cyc_cam")
WO_NODE_INVALID = 0xFFFFFFFF


class Vec3(Structure):
    _fields_ = [("x", c_double), ("y", c_double), ("z", c_double)]


class Quaternion(Structure):
    _fields_ = [("real", c_double), ("imaginary", Vec3)]


class NodeArgument(Structure):
    _fields_ = [("orientation", Quaternion), ("offset", Vec3), ("node", c_uint32)]


class RenderParams(Structure):
    _fields_ = [("width", c_uint32), ("height", c_uint32), ("spp", c_uint32), ("max_depth", c_uint32),
                ("seed", c_uint32), ("mode", c_uint32), ("sample_offset", c_uint32), ("time_sec", c_float)]


class WoRec(Structure):
    _fields_ = [("op", c_uint32), ("u0", c_uint32), ("u1", c_uint32), ("f", c_float * 5)]


class WoMaterial(Structure):
    _fields_ = [("kind", c_uint32), ("albedo", c_float * 3), ("fuzz", c_float), ("ior", c_float),
                ("inv_ior", c_float), ("r0", c_float)]


class WoCamera(Structure):
    _fields_ = [("origin", c_float * 3), ("lower_left", c_float * 3), ("horizontal", c_float * 3),
                ("vertical", c_float * 3), ("u", c_float * 3), ("v", c_float * 3), ("lens_radius", c_float),
                ("pad", c_float * 3)]


class WoFrame(Structure):
    _fields_ = [("width", c_uint32), ("height", c_uint32), ("spp", c_uint32), ("max_depth", c_uint32),
                ("seed", c_uint32), ("mode", c_uint32), ("sample_offset", c_uint32), ("tile_rows", c_uint32),
                ("rank", c_uint32), ("nranks", c_uint32), ("n_recs", c_uint32), ("n_prims", c_uint32),
                ("time_sec", c_float), ("sphere_y", c_float), ("inv_width", c_float), ("inv_height", c_float),
                ("cam", WoCamera), ("band_cycle", c_uint32), ("band_skip", c_uint32)]


assert ctypes.sizeof(Vec3) == 24 and ctypes.sizeof(Quaternion) == 32 and ctypes.sizeof(NodeArgument) == 64
assert ctypes.sizeof(WoRec) == 32 and ctypes.sizeof(WoMaterial) == 32

# Every exported symbol and its signature (restype, argtypes).  tests/ check that the
# library exports exactly these names (the C-ABI declared in include/wololo/*.h).
_R = POINTER(ctypes.c_char)  # opaque Wo_Renderer*
SIGNATURES = {
    # renderer.h (reference API)
    "wo_renderer_new": (c_void_p, [c_void_p, c_char_p, c_size_t]),
    "wo_renderer_del": (None, [c_void_p]),
    "wo_renderer_draw_frame": (None, [c_void_p]),
    "wo_renderer_add_sphere_node": (c_uint32, [c_void_p, c_double]),
    "wo_renderer_add_infinite_planar_partition_node": (c_uint32, [c_void_p, Vec3]),
    "wo_renderer_add_union_of_node": (c_uint32, [c_void_p, NodeArgument, NodeArgument]),
    "wo_renderer_add_intersection_of_node": (c_uint32, [c_void_p, NodeArgument, NodeArgument]),
    "wo_renderer_add_difference_of_node": (c_uint32, [c_void_p, NodeArgument, NodeArgument]),
    "wo_renderer_isroot": (c_bool, [c_void_p, c_uint32]),
    # app.h (reference API + extensions)
    "wo_app_new": (c_void_p, [c_double, c_uint32, c_uint32, c_char_p, c_void_p, c_void_p, c_void_p]),
    "wo_app_run": (c_bool, [c_void_p]),
    "wo_app_swap_scene": (None, [c_void_p, c_void_p]),
    "wo_app_glfw_window": (c_void_p, [c_void_p]),
    "wo_app_window_width": (c_uint32, [c_void_p]),
    "wo_app_window_height": (c_uint32, [c_void_p]),
    "wo_app_time_sec": (c_double, [c_void_p]),
    # renderer_ext.h
    "wo_render_params_default": (None, [POINTER(RenderParams)]),
    "wo_renderer_add_lambertian_material": (c_uint32, [c_void_p, Vec3]),
    "wo_renderer_add_metal_material": (c_uint32, [c_void_p, Vec3, c_double]),
    "wo_renderer_add_dielectric_material": (c_uint32, [c_void_p, c_double]),
    "wo_renderer_set_node_material": (c_bool, [c_void_p, c_uint32, c_uint32]),
    "wo_renderer_set_camera": (None, [c_void_p, Vec3, Vec3, Vec3, c_double, c_double, c_double]),
    "wo_renderer_set_draw_params": (None, [c_void_p, POINTER(RenderParams), c_int]),
    "wo_renderer_render_f32": (c_int, [c_void_p, POINTER(RenderParams), c_void_p]),
    "wo_renderer_render_rows_device": (c_int, [c_void_p, POINTER(RenderParams), c_void_p, c_uint32, c_uint32,
                                               c_uint32, c_void_p, c_void_p]),
    "wo_renderer_count_work": (c_int, [c_void_p, POINTER(RenderParams), c_uint32, c_uint32, c_uint32,
                                       POINTER(c_ulonglong)]),
    "wo_assemble_rows_device": (c_int, [c_void_p, c_void_p, c_uint32, c_uint32, c_uint32, c_uint32, c_void_p]),
    "wo_assemble_rows_device_ex": (c_int, [c_void_p, c_void_p, c_uint32, c_uint32, c_uint32, c_uint32, c_uint32,
                                           c_uint32, c_void_p]),
    "wo_renderer_set_band_weight": (c_int, [c_void_p, c_uint32, c_uint32]),
    "wo_renderer_set_devices": (c_int, [c_void_p, c_int]),
    "wo_renderer_device_count": (c_int, [c_void_p]),
    "wo_renderer_frame_ranks": (c_int, [c_void_p, POINTER(RenderParams)]),
    "wo_renderer_peer_mode": (c_int, [c_void_p, c_int]),
    "wo_renderer_render_frame_device": (c_int, [c_void_p, POINTER(RenderParams), c_void_p, c_void_p]),
    "wo_renderer_take_segments": (c_int, [c_void_p, POINTER(c_ulonglong)]),
    "wo_renderer_finish": (c_int, [c_void_p]),
    "wo_renderer_last_frame": (POINTER(c_float), [c_void_p, POINTER(c_uint32), POINTER(c_uint32)]),
    "wo_renderer_last_frame_bgra8": (POINTER(c_uint32), [c_void_p, POINTER(c_uint32), POINTER(c_uint32)]),
    "wo_renderer_set_map_float": (None, [c_void_p, c_int]),
    "wo_renderer_set_frame_stamps": (c_int, [c_void_p, c_int]),
    "wo_renderer_frame_stamps": (c_int, [c_void_p, POINTER(c_double), c_int]),
    "wo_srgb8_thresholds": (None, [POINTER(c_float)]),
    "wo_srgb8_encode_device": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "wo_srgb8_encode_host": (None, [c_void_p, c_void_p, c_size_t]),
    "wo_renderer_set_progressive": (None, [c_void_p, c_int]),
    "wo_renderer_accumulated_spp": (c_uint32, [c_void_p]),
    "wo_renderer_render_accumulate": (c_int, [c_void_p, POINTER(RenderParams), c_void_p, c_int]),
    "wo_renderer_compile": (c_int, [c_void_p]),
    "wo_renderer_program": (POINTER(WoRec), [c_void_p, POINTER(c_uint32), POINTER(c_uint32)]),
    "wo_renderer_materials": (POINTER(WoMaterial), [c_void_p, POINTER(c_uint32)]),
    "wo_renderer_frame_desc": (c_int, [c_void_p, POINTER(RenderParams), c_uint32, c_uint32, c_uint32,
                                       POINTER(WoFrame)]),
    "wo_renderer_set_jit": (None, [c_void_p, c_int]),
    "wo_renderer_set_tracer": (None, [c_void_p, c_int]),
    "wo_renderer_trace_path": (c_char_p, [c_void_p]),
    "wo_renderer_set_jit_async": (None, [c_void_p, c_int]),
    "wo_renderer_jit_pending": (c_int, [c_void_p]),
    "wo_renderer_prepare": (c_int, [c_void_p]),
    "wo_renderer_jit_source": (c_void_p, [c_void_p]),
    "wo_jit_compile_check": (c_int, [c_char_p, c_char_p, c_char_p, c_size_t]),
    "wo_jit_code_resources": (c_int, [c_char_p, c_char_p, POINTER(ctypes.c_uint32), c_char_p, ctypes.c_size_t]),
    "wo_jit_code_object": (ctypes.c_longlong, [c_char_p, c_char_p, POINTER(c_int), POINTER(c_double), c_char_p,
                                               c_char_p, c_size_t]),
    "wo_renderer_jit_info": (c_int, [c_void_p, POINTER(c_double)]),
    "wo_renderer_lanes_info": (c_int, [c_void_p, POINTER(c_uint32)]),
    "wo_renderer_kernel_info": (c_int, [c_void_p, c_char_p, POINTER(c_uint32)]),
    "wo_free": (None, [c_void_p]),
    "wo_renderer_node_count": (c_size_t, [c_void_p]),
    "wo_renderer_name": (c_char_p, [c_void_p]),
    "wo_renderer_device": (c_int, [c_void_p]),
    "wo_renderer_last_error": (c_char_p, []),
    "wo_renderer_clear_error": (None, []),
    "wo_version": (c_char_p, []),
    "wo_abi_layout": (c_size_t, [c_char_p, c_char_p]),
    "wo_hip_device_count": (c_int, []),
    "wo_hip_runtime_version": (c_int, []),
    "wo_fastmath_check": (c_int, [c_int, c_uint32, c_uint32, POINTER(c_ulonglong), POINTER(c_uint32)]),
}

_lib = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Load libwololo.so (raises if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"libwololo.so not found at {p}; build it with `python -c 'import __graft_entry__ as g; "
                           f"g.build()'` or `make -C csgrenderer_amd/csrc`")
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        if os.environ.get("WOLOLO_LIB") and not hasattr(lib, name):
            continue  # an older build under A/B measurement: bind what it has
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def vec3(x, y, z) -> Vec3:
    return Vec3(float(x), float(y), float(z))


def quat_identity() -> Quaternion:
    return Quaternion(1.0, Vec3(0.0, 0.0, 0.0))


def arg(node: int, offset=(0.0, 0.0, 0.0), orientation: Quaternion | None = None) -> NodeArgument:
    return NodeArgument(orientation or quat_identity(), vec3(*offset), int(node))


def last_error() -> str:
    e = load().wo_renderer_last_error()
    return e.decode() if e else ""


def clear_error():
    load().wo_renderer_clear_error()


class WololoError(RuntimeError):
    pass


class Renderer:
    """Thin owner of a Wo_Renderer* (all calls go straight to the C library)."""

    def __init__(self, name: str = "py", max_nodes: int = 1024, app: int | None = None):
        self.lib = load()
        self.ptr = self.lib.wo_renderer_new(app, name.encode(), max_nodes)
        if not self.ptr:
            raise WololoError(f"wo_renderer_new failed: {last_error()}")

    def close(self):
        if self.ptr:
            self.lib.wo_renderer_del(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- nodes (reference API) ----
    def _check(self, n: int) -> int:
        if n == WO_NODE_INVALID:
            raise WololoError(last_error())
        return n

    def sphere(self, radius: float) -> int:
        return self._check(self.lib.wo_renderer_add_sphere_node(self.ptr, float(radius)))

    def halfspace(self, normal) -> int:
        return self._check(self.lib.wo_renderer_add_infinite_planar_partition_node(self.ptr, vec3(*normal)))

    def union(self, a: NodeArgument, b: NodeArgument) -> int:
        return self._check(self.lib.wo_renderer_add_union_of_node(self.ptr, a, b))

    def intersection(self, a: NodeArgument, b: NodeArgument) -> int:
        return self._check(self.lib.wo_renderer_add_intersection_of_node(self.ptr, a, b))

    def difference(self, a: NodeArgument, b: NodeArgument) -> int:
        return self._check(self.lib.wo_renderer_add_difference_of_node(self.ptr, a, b))

    def isroot(self, n: int) -> bool:
        return bool(self.lib.wo_renderer_isroot(self.ptr, n))

    # ---- extensions ----
    def lambertian(self, albedo) -> int:
        return self.lib.wo_renderer_add_lambertian_material(self.ptr, vec3(*albedo))

    def metal(self, albedo, fuzz: float) -> int:
        return self.lib.wo_renderer_add_metal_material(self.ptr, vec3(*albedo), float(fuzz))

    def dielectric(self, ior: float) -> int:
        return self.lib.wo_renderer_add_dielectric_material(self.ptr, float(ior))

    def set_material(self, leaf: int, mat: int):
        if not self.lib.wo_renderer_set_node_material(self.ptr, leaf, mat):
            raise WololoError(f"set_node_material({leaf}, {mat}) rejected")

    def set_camera(self, look_from, look_at, vup=(0, 1, 0), vfov=90.0, aperture=0.0, focus_dist=1.0):
        self.lib.wo_renderer_set_camera(self.ptr, vec3(*look_from), vec3(*look_at), vec3(*vup), float(vfov),
                                        float(aperture), float(focus_dist))

    def compile(self) -> int:
        n = self.lib.wo_renderer_compile(self.ptr)
        if n < 0:
            raise WololoError(last_error())
        return n

    def program(self):
        """(records ctypes array, n_prims) of the compiled scene."""
        nr, npr = c_uint32(0), c_uint32(0)
        p = self.lib.wo_renderer_program(self.ptr, ctypes.byref(nr), ctypes.byref(npr))
        if not p:
            raise WololoError(last_error())
        arr = (WoRec * max(nr.value, 1))()
        if nr.value:
            ctypes.memmove(arr, p, ctypes.sizeof(WoRec) * nr.value)
        return arr, nr.value, npr.value

    def materials(self):
        n = c_uint32(0)
        p = self.lib.wo_renderer_materials(self.ptr, ctypes.byref(n))
        arr = (WoMaterial * max(n.value, 1))()
        ctypes.memmove(arr, p, ctypes.sizeof(WoMaterial) * n.value)
        return arr, n.value

    def jit_source(self) -> str | None:
        p = self.lib.wo_renderer_jit_source(self.ptr)
        if not p:
            return None
        try:
            return ctypes.string_at(p).decode()
        finally:
            self.lib.wo_free(p)

    def jit_info(self):
        """(origin, seconds) of the specialised kernel: origin "process" / "disk" / "compiled", or None."""
        sec = c_double(0.0)
        o = self.lib.wo_renderer_jit_info(self.ptr, ctypes.byref(sec))
        return (None if o < 0 else JIT_ORIGINS[o]), sec.value

    def lanes_info(self):
        """The lane tracer's BVH: {"nodes", "depth", "top", "always", "kind"} ("kind": the kernel
        form of the last path launch, trace_kernels.hip PathKind), or None if not on the lane tracer."""
        out = (c_uint32 * 5)()
        if self.lib.wo_renderer_lanes_info(self.ptr, out) < 0:
            return None
        return dict(zip(("nodes", "depth", "top", "always", "kind"), list(out)))

    def set_jit(self, mode: int):
        self.lib.wo_renderer_set_jit(self.ptr, int(mode))

    def set_tracer(self, tracer):
        """TRACER_AUTO / _INTERPRETER / _JIT / _LANES, or the names "auto", "interpreter", "jit", "lanes"."""
        if isinstance(tracer, str):
            tracer = TRACERS[tracer]
        self.lib.wo_renderer_set_tracer(self.ptr, int(tracer))

    def set_jit_async(self, on: bool):
        self.lib.wo_renderer_set_jit_async(self.ptr, 1 if on else 0)

    def jit_pending(self) -> bool:
        return bool(self.lib.wo_renderer_jit_pending(self.ptr))

    def kernel_info(self):
        """The last launch's path kernel as loaded (renderer_ext.h wo_renderer_kernel_info):
        {"key", "kind", "scratch_bytes", "vgprs", "lds_bytes"}, or None before a path launch."""
        key = ctypes.create_string_buffer(65)
        out = (c_uint32 * 4)()
        if self.lib.wo_renderer_kernel_info(self.ptr, key, out) != 0:
            return None
        return {"key": key.value.decode(), "kind": int(out[0]), "scratch_bytes": int(out[1]),
                "vgprs": int(out[2]), "lds_bytes": int(out[3])}

    def prepare(self):
        """Compile, upload and load the scene's kernels now, waiting for a background
        compile (renderer_ext.h wo_renderer_prepare)."""
        if self.lib.wo_renderer_prepare(self.ptr) != 0:
            raise WololoError(last_error())

    def trace_path(self) -> str:
        return self.lib.wo_renderer_trace_path(self.ptr).decode()

    def frame_desc(self, params: RenderParams, tile_rows=16, rank=0, nranks=1) -> WoFrame:
        fr = WoFrame()
        if self.lib.wo_renderer_frame_desc(self.ptr, ctypes.byref(params), tile_rows, rank, nranks,
                                           ctypes.byref(fr)):
            raise WololoError(last_error())
        return fr

    def render(self, params: RenderParams):
        """Full frame to host; returns a float32 numpy array (H, W, 4)."""
        import numpy as np
        out = np.empty((params.height, params.width, 4), dtype=np.float32)
        if self.lib.wo_renderer_render_f32(self.ptr, ctypes.byref(params), out.ctypes.data_as(c_void_p)):
            raise WololoError(last_error())
        return out

    def render_accumulate(self, params: RenderParams, reset: bool = False):
        """params.spp more samples into the progressive accumulation; returns (mean image, total spp)."""
        import numpy as np
        out = np.empty((params.height, params.width, 4), dtype=np.float32)
        n = self.lib.wo_renderer_render_accumulate(self.ptr, ctypes.byref(params), out.ctypes.data_as(c_void_p),
                                                   1 if reset else 0)
        if n < 0:
            raise WololoError(last_error())
        return out, n

    def draw_frame(self):
        """wo_renderer_draw_frame (pipelined: presents the previous frame)."""
        self.lib.wo_renderer_draw_frame(self.ptr)

    def set_devices(self, n: int) -> int:
        """Split every frame over n ranks (renderer_ext.h wo_renderer_set_devices)."""
        rc = self.lib.wo_renderer_set_devices(self.ptr, int(n))
        if rc < 0:
            raise WololoError(last_error())
        return rc

    def device_count(self) -> int:
        return int(self.lib.wo_renderer_device_count(self.ptr))

    def frame_ranks(self, params: RenderParams) -> int:
        """Ranks a frame with these parameters is split over (wo_renderer_frame_ranks)."""
        return int(self.lib.wo_renderer_frame_ranks(self.ptr, ctypes.byref(params)))

    def peer_mode(self, rank: int) -> str | None:
        """How rank `rank`'s share reaches rank 0: "same", "dma" or "staged" (None for rank 0)."""
        m = self.lib.wo_renderer_peer_mode(self.ptr, int(rank))
        return None if m < 0 else PEER_MODES[m]

    def render_frame_device(self, params: RenderParams, d_frame: int, stream: int = 0):
        """Whole frame over the renderer's ranks into device memory (wo_renderer_render_frame_device)."""
        if self.lib.wo_renderer_render_frame_device(self.ptr, ctypes.byref(params), c_void_p(d_frame),
                                                    c_void_p(stream or None)):
            raise WololoError(last_error())

    def take_segments(self) -> int:
        """Segments traced by render_frame_device frames since the last call (all ranks)."""
        t = c_ulonglong(0)
        if self.lib.wo_renderer_take_segments(self.ptr, ctypes.byref(t)):
            raise WololoError(last_error())
        return int(t.value)

    def finish(self):
        if self.lib.wo_renderer_finish(self.ptr):
            raise WololoError(last_error())

    def last_frame(self):
        """Copy of the last presented frame (H, W, 4) or None."""
        import numpy as np
        w, h = c_uint32(0), c_uint32(0)
        p = self.lib.wo_renderer_last_frame(self.ptr, ctypes.byref(w), ctypes.byref(h))
        if not p:
            return None
        return np.ctypeslib.as_array(p, shape=(h.value * w.value * 4,)).reshape(h.value, w.value, 4).copy()

    def last_frame_bgra8(self):
        """Copy of the last presented frame's present encode, (H, W) uint32 B8G8R8A8 sRGB, or None."""
        import numpy as np
        w, h = c_uint32(0), c_uint32(0)
        p = self.lib.wo_renderer_last_frame_bgra8(self.ptr, ctypes.byref(w), ctypes.byref(h))
        if not p:
            return None
        return np.ctypeslib.as_array(p, shape=(h.value * w.value,)).reshape(h.value, w.value).copy()

    def set_map_float(self, every_frame: bool):
        """Map every presented frame's float pixels back (True) or only when last_frame() asks (default)."""
        self.lib.wo_renderer_set_map_float(self.ptr, 1 if every_frame else 0)

    def set_frame_stamps(self, on: bool):
        if self.lib.wo_renderer_set_frame_stamps(self.ptr, 1 if on else 0):
            raise WololoError(last_error())

    def frame_stamps(self):
        """Logged pipeline stamps, a list of (render_begin, render_end, mapback_end) ms per presented frame."""
        buf = (c_double * (3 * 256))()
        n = self.lib.wo_renderer_frame_stamps(self.ptr, buf, 256)
        if n < 0:
            raise WololoError(last_error())
        return [tuple(buf[3 * i:3 * i + 3]) for i in range(n)]

    def set_draw_params(self, params: RenderParams, pin_time: bool = True):
        self.lib.wo_renderer_set_draw_params(self.ptr, ctypes.byref(params), 1 if pin_time else 0)

    def set_progressive(self, on: bool):
        self.lib.wo_renderer_set_progressive(self.ptr, 1 if on else 0)

    def accumulated_spp(self) -> int:
        return int(self.lib.wo_renderer_accumulated_spp(self.ptr))

    def count_work(self, params: RenderParams, tile_rows: int = 4, rank: int = 0, nranks: int = 1) -> dict:
        """Executed-work counters of one frame (wo_renderer_count_work), by WORK_KINDS name."""
        c = (c_ulonglong * len(WORK_KINDS))()
        if self.lib.wo_renderer_count_work(self.ptr, ctypes.byref(params), tile_rows, rank, nranks, c):
            raise WololoError(last_error())
        return dict(zip(WORK_KINDS, (int(v) for v in c)))

    def set_band_weight(self, cycle: int, skip: int):
        """Weighted row bands of multi-rank frames: rank 0 sits out `skip` of every `cycle` rounds."""
        if self.lib.wo_renderer_set_band_weight(self.ptr, cycle, skip):
            raise WololoError(last_error())

    def render_rows_device(self, params: RenderParams, d_out: int, tile_rows: int, rank: int, nranks: int,
                           stream: int = 0, d_segments: int = 0):
        if self.lib.wo_renderer_render_rows_device(self.ptr, ctypes.byref(params), c_void_p(d_out), tile_rows, rank,
                                                   nranks, c_void_p(stream or None),
                                                   c_void_p(d_segments or None)):
            raise WololoError(last_error())


def render_params(width=256, height=256, spp=1, max_depth=8, seed=0, mode=MODE_UBERSHADER_RT1, sample_offset=0,
                  time_sec=0.0) -> RenderParams:
    return RenderParams(width, height, spp, max_depth, seed, mode, sample_offset, float(time_sec))


def assemble_rows_device(d_gathered: int, d_frame: int, width: int, height: int, tile_rows: int, nranks: int,
                         stream: int = 0, band=(0, 0)):
    """Un-interleave the gathered rank buffers; `band` = (cycle, skip) of weighted bands."""
    lib = load()
    if lib.wo_assemble_rows_device_ex(c_void_p(d_gathered), c_void_p(d_frame), width, height, tile_rows, nranks,
                                      band[0], band[1], c_void_p(stream or None)):
        raise WololoError(last_error())


def srgb8_thresholds():
    """The present encode's 255 thresholds (float32 numpy array)."""
    import numpy as np
    t = (c_float * 255)()
    load().wo_srgb8_thresholds(t)
    return np.frombuffer(t, dtype=np.float32).copy()


def srgb8_encode_host(rgba):
    """(..., 4) float32 RGBA -> (...) uint32 B8G8R8A8 sRGB, the library's host encode."""
    import numpy as np
    a = np.ascontiguousarray(rgba, dtype=np.float32)
    out = np.empty(a.shape[:-1], dtype=np.uint32)
    load().wo_srgb8_encode_host(a.ctypes.data_as(c_void_p), out.ctypes.data_as(c_void_p), out.size)
    return out


def srgb8_encode_device(d_rgba: int, d_bgra8: int, pixels: int, stream: int = 0):
    if load().wo_srgb8_encode_device(c_void_p(d_rgba), c_void_p(d_bgra8), pixels, c_void_p(stream or None)):
        raise WololoError(last_error())


def abi_layout(type_name: str, field: str | None = None) -> int:
    """sizeof / offsetof as the C library was compiled (wo_abi_layout); -1 if unknown."""
    v = load().wo_abi_layout(type_name.encode(), field.encode() if field else None)
    return -1 if v == ctypes.c_size_t(-1).value else int(v)


JIT_ORIGINS = ("process", "disk", "compiled")
PEER_MODES = ("same", "dma", "staged")  # wo_dev.h WO_PEER_*


def jit_code_object(src: str, arch: str = "gfx950"):
    """(size, origin, seconds, key) of the specialised kernel's code object (wo_jit_code_object)."""
    err = ctypes.create_string_buffer(4096)
    key = ctypes.create_string_buffer(65)
    org, sec = c_int(-1), c_double(0.0)
    n = load().wo_jit_code_object(src.encode(), arch.encode(), ctypes.byref(org), ctypes.byref(sec), key, err,
                                  len(err))
    if n < 0:
        raise WololoError(err.value.decode(errors="replace"))
    return int(n), JIT_ORIGINS[org.value], sec.value, key.value.decode()


def jit_code_resources(src: str, arch: str = "gfx950"):
    """(scratch bytes per lane, static LDS bytes) of the specialised kernel's code object, from
    its kernel descriptor (wo_jit_code_resources; no GPU needed)."""
    err = ctypes.create_string_buffer(4096)
    out = (ctypes.c_uint32 * 2)()
    if load().wo_jit_code_resources(src.encode(), arch.encode(), out, err, len(err)):
        raise WololoError(err.value.decode(errors="replace"))
    return int(out[0]), int(out[1])


def jit_compile_check(src: str, arch: str = "gfx950") -> str:
    """Compile generated source with hiprtc (no GPU needed); '' on success, else the log."""
    err = ctypes.create_string_buffer(4096)
    rc = load().wo_jit_compile_check(src.encode(), arch.encode(), err, len(err))
    return "" if rc == 0 else err.value.decode(errors="replace")


BAND_CYCLE_MAX = 65536  # wo_scene.h WO_BAND_CYCLE_MAX


def _weighted(nranks, band):
    return nranks >= 2 and 0 < band[1] < band[0] <= BAND_CYCLE_MAX


def band_global(lb: int, rank: int, nranks: int, band=(0, 0)) -> int:
    """Mirror of wo_band_global() (wo_scene.h): the frame band of a rank's local band."""
    if not _weighted(nranks, band):
        return lb * nranks + rank
    cycle, skip = band
    full = cycle - skip
    per = full if rank == 0 else cycle
    c, j = divmod(lb, per)
    p = j * nranks + rank if j < full else full * nranks + (j - full) * (nranks - 1) + rank - 1
    return c * (cycle * nranks - skip) + p


def rank_bands(height: int, tile_rows: int, rank: int, nranks: int, band=(0, 0)) -> int:
    """Mirror of wo_rank_tile_count_ex() (wo_scene.h)."""
    tiles = (height + tile_rows - 1) // tile_rows
    if not _weighted(nranks, band):
        return (tiles - rank + nranks - 1) // nranks if rank < tiles else 0
    cycle, skip = band
    per = cycle - skip if rank == 0 else cycle
    c, rem = divmod(tiles, cycle * nranks - skip)
    return c * per + sum(1 for j in range(per) if band_global(j, rank, nranks, band) < rem)


def default_band(nranks: int):
    """The row-band weighting bench.py gives an N-rank frame: rank 0 (which also
    receives the gather, assembles and presents) sits out one round of bands in
    every `cycle`.  tools/root_step.py, csg32 1080p64, N = 8: 0:0 6.21x, 8:1 6.37x,
    12:1 6.44x; N = 4: 0:0 3.33x, 16:1 3.59x; N = 2: 0:0 1.89x, 32:1 1.92x.  Heavier
    scenes want a lighter skip (rank 0's extra work is the same milliseconds).  Round 5
    (camera-ray waves make the shares shorter, rank 0's extra work is not): N = 8 without
    the present map-back, csg32 10:1 6.69x / 5:1 6.87x, csg32_nested 7.29 / 7.66x, RTIOW
    7.45 / 7.36x (profiles/r05_root_step_nomap_n8.log)."""
    if nranks >= 8:
        return (5, 1)
    if nranks >= 4:
        return (16, 1)
    if nranks >= 2:
        return (32, 1)
    return (0, 0)


def local_rows(height: int, tile_rows: int, nranks: int, band=(0, 0)) -> int:
    """Mirror of wo_rank_local_rows_ex() (wo_scene.h)."""
    t = [rank_bands(height, tile_rows, r, nranks, band) for r in range(min(nranks, 2))]
    return max(t) * tile_rows


def global_row(lrow: int, tile_rows: int, rank: int, nranks: int, band=(0, 0)) -> int:
    lt = lrow // tile_rows
    return band_global(lt, rank, nranks, band) * tile_rows + (lrow - lt * tile_rows)
