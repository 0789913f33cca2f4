"""csgrenderer_amd -- MI355X-native wololo CSG renderer.

The product is ``lib/libwololo.so`` (C host + HIP kernels for gfx950, built from
``csrc/``); ``wololo`` binds its C ABI, ``scenes`` builds the benchmark scenes
through that API.
"""
from . import wololo  # noqa: F401
from .build import build_library  # noqa: F401

__all__ = ["wololo", "build_library"]
