"""Build helpers: compile libwololo.so (HIP for gfx950 + C host) in-tree."""
from __future__ import annotations

import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")


def build_library(jobs: int = 8, quiet: bool = False) -> str:
    env = dict(os.environ)
    env.setdefault("ARCH", "gfx950")
    subprocess.run(["make", "-C", CSRC, f"-j{jobs}"], check=True, env=env,
                   stdout=subprocess.DEVNULL if quiet else None)
    lib = os.path.join(PKG_DIR, "lib", "libwololo.so")
    if not os.path.exists(lib):
        raise RuntimeError("build finished but libwololo.so is missing")
    return lib
