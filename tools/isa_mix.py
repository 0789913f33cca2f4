#!/usr/bin/env python3
"""Static instruction mix of a scene's generated kernel per path-loop section (the
WO_ISA_MARKS markers: cam_begin, collect_begin/end, shade_begin/end, take_begin), by
class: VALU arithmetic (v_add/mul/fma/...), VALU select/move (v_cndmask, v_mov),
VALU compare, SALU, LDS, VMEM, branch/exec.  Diagnostic for where the kernel's
non-arithmetic instructions sit.

    python tools/isa_mix.py csg32 [-D WO_...]
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def klass(op):
    if op.startswith("v_cndmask") or op.startswith("v_mov") or op.startswith("v_readlane") or op.startswith("v_writelane") \
            or op.startswith("v_readfirstlane"):
        return "valu_select_move"
    if op.startswith("v_cmp"):
        return "valu_compare"
    if op.startswith(("v_add", "v_sub", "v_mul", "v_fma", "v_fmac", "v_mad", "v_max", "v_min", "v_rsq", "v_rcp",
                      "v_sqrt", "v_med3", "v_pk_", "v_trunc", "v_floor", "v_rndne", "v_fract", "v_ldexp", "v_cvt",
                      "v_div", "v_exp", "v_log", "v_sin", "v_cos", "v_frexp")):
        return "valu_arith"
    if op.startswith("v_"):
        return "valu_bit_int"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op.startswith(("s_cbranch", "s_branch", "s_and_saveexec", "s_or_saveexec", "s_andn2_saveexec", "s_xor_b64 exec")):
        return "branch_exec"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scene")
    ap.add_argument("-D", action="append", default=[])
    a = ap.parse_args()
    d = tempfile.mkdtemp()
    s_path = os.path.join(d, "k.s")
    cmd = [sys.executable, os.path.join(ROOT, "tools", "jit_isa.py"), a.scene, "-D", "WO_ISA_MARKS", "--keep", s_path]
    for x in a.D:
        cmd += ["-D", x]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)
    sec = "prologue"
    mix = collections.defaultdict(collections.Counter)
    for line in open(s_path):
        m = re.search(r";WOMARK (\w+)", line)
        if m:
            sec = {"cam_begin": "camera jobs", "collect_begin": "collect", "collect_end": "sweep",
                   "shade_begin": "shade", "shade_end": "ring / accumulate", "take_begin": "take"}.get(m.group(1), m.group(1))
            continue
        t = line.strip()
        if not t or t.startswith((";", ".", "_")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith("s_waitcnt") or op.startswith("s_nop"):
            continue
        mix[sec][klass(op)] += 1
    classes = ["valu_arith", "valu_compare", "valu_select_move", "valu_bit_int", "salu", "branch_exec", "lds", "vmem",
               "smem", "other"]
    print(f"{'section':<20}" + "".join(f"{c:>17}" for c in classes) + f"{'total':>8}")
    for s, c in mix.items():
        print(f"{s:<20}" + "".join(f"{c[k]:>17}" for k in classes) + f"{sum(c.values()):>8}")


if __name__ == "__main__":
    main()
