#!/usr/bin/env python3
"""Mismatches of the fast correctly rounded math per binade (diagnostic).
which 0: sqrt_cr, 1: rcp_cr, each against the exact definition of correct rounding.
    python tools/fastmath_scan.py [which ...]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from csgrenderer_amd import wololo as wl  # noqa: E402

lib = wl.load()
for which in [int(a) for a in sys.argv[1:]] or [0, 1]:
    rows = []
    total = 0
    for e in range(1, 255):
        lo, hi = e << 23, ((e + 1) << 23) - 1
        bad, first = ctypes.c_ulonglong(0), ctypes.c_uint32(0)
        lib.wo_fastmath_check(which, lo, hi, ctypes.byref(bad), ctypes.byref(first))
        total += bad.value
        if bad.value:
            rows.append((e - 127, bad.value, hex(first.value)))
    print("which", which, "total mismatches", total, "first binades:", rows[:6], "last:", rows[-3:], flush=True)
