"""Scene-specialised kernels (csrc/scene_jit.c): the generated HIP source compiles
for gfx950 with hiprtc (no GPU needed) and mirrors the compiled program (CPU)."""
import math
import re

import numpy as np
import pytest

from csgrenderer_amd import scenes
from csgrenderer_amd import wololo as wl


_SINGLE_RE = r"wodev::(sphere_interval|sphere_interval_bd|sphere_need|halfspace_interval|halfspace_axis_interval|halfspace_axis_dist)\("


def _leaf_calls(src):
    """(single-leaf interval calls, slab face-pair calls) in the generated source: a
    sphere with literal constants ends in sphere_interval_bd, or is a lone sphere
    tested with sphere_need; an axis face ends in halfspace_axis_dist; two opposite
    faces of a slab are one axis_pair_meet."""
    return len(re.findall(_SINGLE_RE, src)), len(re.findall(r"wodev::axis_pair_meet(_d)?\(", src))


def test_generated_sources_compile_for_gfx950(hostonly):
    """The three forms the generator picks by scene, each compiled by hiprtc for gfx950:
    the event list with the scene compiler's BOUND records as the culling structure
    (csg256_balanced: > 64 primitives in a shallow tree), the event list collected over
    the CSG tree with relevance groups (csg32_nested: a general root over <= 64
    primitives, two boxes), and term mode (csg32: a union of <= 2-literal conjunctions)."""
    # BOUND records: wave-level tests only for subtrees of >= 4 leaves and not around a
    # lone primitive (its member skip is the cheaper test)
    r = wl.Renderer("jit", max_nodes=4096)
    scenes.build("csg256_balanced", r)
    prog, nrec, nprim = r.program()
    src = r.jit_source()
    nleaf = sum(1 for i in range(nrec) if prog[i].op in (wl.WO_LEAF_SPHERE, wl.WO_LEAF_HALFSPACE))
    nsingle, npair = _leaf_calls(src)
    assert nsingle + 2 * npair == 2 * nleaf  # every leaf in both collect passes

    def lone(i):
        return prog[i + 1].op == wl.WO_OP_PRIM and i + 2 + prog[i + 1].u0 == prog[i].u0

    nb = sum(1 for i in range(nrec) if prog[i].op == wl.WO_OP_BOUND and prog[i].u1 >= 4 and not lone(i))
    assert 0 < nb < sum(1 for i in range(nrec) if prog[i].op == wl.WO_OP_BOUND)
    assert len(re.findall(r"if \(__ballot\(!miss\) == 0ull\)", src)) == nb
    assert "// group" not in src and "kUTerm" in src  # the union count of its pair terms
    m = re.search(r"kOrdPc\[(\d+)\] = \{([^}]*)\}", src)
    assert int(m.group(1)) == nprim
    pcs = [int(x.strip().rstrip("u")) for x in m.group(2).split(",")]
    assert pcs == [i for i in range(nrec) if prog[i].op == wl.WO_OP_PRIM]
    log = wl.jit_compile_check(src, "gfx950")
    assert log == "", log
    r.close()
    # the tree collect with relevance groups (a general tree with truth tables): one
    # wave-level test per group of >= 4 primitives, no BOUND record or spatial group
    # tested; every leaf still intersected in both passes (none of csg32_nested's is
    # outside its relevance box); the two boxes' axis faces on the fast path
    r = wl.Renderer("jit", max_nodes=4096)
    scenes.build("csg32_nested", r)
    prog, nrec, nprim = r.program()
    src = r.jit_source()
    nleaf = sum(1 for i in range(nrec) if prog[i].op in (wl.WO_LEAF_SPHERE, wl.WO_LEAF_HALFSPACE))
    ngroups = len(re.findall(r"// relevance group \d+ \((\d+) primitives\)", src))  # the first pass tests them
    assert ngroups >= 2 and "// BOUND" not in src and "// group" not in src
    first = src[:src.index('WO_MARK("collect_end")')]
    assert len(set(re.findall(r"// primitive (\d+)", first))) == nprim
    assert len(re.findall(r"if \(__ballot\(!miss\) == 0ull\)", src)) == ngroups
    nsingle, npair = _leaf_calls(src)
    # the first pass and a re-collect copy per sweep form (the batch sweep's and the
    # event loop's, one of which WO_SWEEP_BATCH compiles)
    npass = 3 if "#if WO_SWEEP_BATCH" in src else 2
    assert npair >= npass * 6  # two boxes: three face pairs each, in every pass
    assert nsingle + 2 * npair == npass * nleaf
    naxis = sum(1 for i in range(nrec) if prog[i].op == wl.WO_LEAF_HALFSPACE and prog[i].u1 != 0)
    assert naxis >= 12
    assert len(re.findall(r"wodev::halfspace_axis_(interval|dist)\(", src)) + 2 * npair == npass * naxis
    assert "wodev::LdsWindow win" in src and "WO_EVAL_BEGIN" in src  # the LDS event list, a general root
    assert wl.jit_compile_check(src, "gfx950") == ""
    r.close()
    # the term form (the root is a union of <= 2-literal conjunctions): every leaf still
    # intersected once per pass, each term once per pass, no event list, no sweep
    r = wl.Renderer("jit", max_nodes=4096)
    scenes.build("csg32", r)
    prog, nrec, nprim = r.program()
    src = r.jit_source()
    nleaf = sum(1 for i in range(nrec) if prog[i].op in (wl.WO_LEAF_SPHERE, wl.WO_LEAF_HALFSPACE))
    m = re.search(r"// term mode: (\d+) terms", src)
    assert m, "csg32 takes the term form"
    nterms = int(m.group(1))
    assert nterms == 14  # 9 pairs (3 unions of two, 3 differences, 3 lenses) + crater + rounded cube ... as terms
    assert len(re.findall(r"\{  // term: ", src)) == 2 * nterms
    assert "wodev::LdsWindow win" not in src and "WO_EVAL_BEGIN" not in src and "#define WO_JIT_LDS_EVENTS 0" in src
    nsingle, npair = _leaf_calls(src)
    assert npair >= 2 * 6  # the slab and the cube
    assert nsingle + 2 * npair == 2 * nleaf
    assert wl.jit_compile_check(src, "gfx950") == ""
    r.close()


def test_literals_round_trip(hostonly):
    """Leaf parameters are emitted as exact fp32 bit patterns (s_mov_b32 immediates)."""
    r = wl.Renderer("lit", max_nodes=8)
    s = r.sphere(0.1)
    h = r.halfspace((0.3, -0.7, 0.2))
    r.union(wl.arg(s, (1.0 / 3.0, 2.0 / 7.0, -1e-7)), wl.arg(h, (0.1, 0.2, 0.3)))
    prog, nrec, _ = r.program()
    src = r.jit_source()
    # scalar moves, or literal operands of the VALU instructions that use them
    imms = {int(x, 16) for x in re.findall(r"(?:s_mov_b32 %\d|v_\w+ %0), 0x([0-9a-f]{8})", src)}
    for i in range(nrec):
        if prog[i].op in (wl.WO_LEAF_SPHERE, wl.WO_LEAF_HALFSPACE):
            # axis-aligned half-spaces carry only h as an SGPR constant (s is a literal)
            ks = [3] if prog[i].op == wl.WO_LEAF_HALFSPACE and prog[i].u1 else range(4)
            for k in ks:
                bits = int(np.array(prog[i].f[k], dtype=np.float32).view(np.uint32))
                assert bits in imms, prog[i].f[k]
    assert wl.jit_compile_check(src) == ""
    r.close()


def test_empty_scene_has_no_source(hostonly):
    r = wl.Renderer("e", max_nodes=2)
    assert r.jit_source() is None
    r.close()


def test_member_skip_guards(hostonly):
    """Members after a primitive's first are guarded by a wave-level emptiness test
    (scene_jit.c gen_members): one guard per later member in each collect pass.
    Exact: a met interval only narrows."""
    guard = "if (__ballot(!(iv.a > iv.b)) != 0ull)"
    r = wl.Renderer("skip", max_nodes=4096)
    scenes.build("csg32", r)
    prog, nrec, _ = r.program()
    src = r.jit_source()
    pair_members = len(re.findall(r"wodev::axis_pair_meet(_d)?\(", src))  # a pair is one member step
    singles = len(re.findall(r"wodev::(sphere_interval|sphere_interval_bd|sphere_need|halfspace_interval|halfspace_axis_interval|halfspace_axis_dist)\(", src))
    nprims_emitted = 2 * sum(1 for i in range(nrec) if prog[i].op == wl.WO_OP_PRIM)
    assert src.count(guard) == singles + pair_members - nprims_emitted > 0
    r.close()


_CHILD = r"""
import json, sys
sys.path.insert(0, {root!r})
from csgrenderer_amd import wololo as wl
src = open({src!r}).read()
n, origin, sec, key = wl.jit_code_object(src, "gfx950")
print(json.dumps({{"n": n, "origin": origin, "sec": sec, "key": key}}))
"""


def _child(tmp_path, src_text, env_extra=None):
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sp = tmp_path / f"src{abs(hash(src_text)) % 10**8}.hip"
    sp.write_text(src_text)
    env = dict(os.environ, WOLOLO_JIT_CACHE=str(tmp_path / "cache"))
    env.pop("WOLOLO_JIT_FLAGS", None)
    env.update(env_extra or {})
    out = subprocess.run([sys.executable, "-c", _CHILD.format(root=root, src=str(sp))], env=env, check=True,
                         capture_output=True, text=True, timeout=300).stdout
    return json.loads(out.strip().splitlines()[-1])


def test_persistent_code_object_cache(hostonly, tmp_path, monkeypatch):
    """The specialised kernel's code object is cached on disk under the SHA-256 of its
    inputs: a second process loads it instead of compiling; a changed scene or a changed
    compile flag misses; a corrupt entry is a miss and is rewritten."""
    import hashlib
    import struct
    r = wl.Renderer("cache", max_nodes=64)
    a = r.sphere(0.5)
    b = r.sphere(0.3)
    r.difference(wl.arg(a), wl.arg(b, (0.2, 0.0, 0.0)))
    src = r.jit_source()
    r.sphere(0.25)  # another root: another scene
    src2 = r.jit_source()
    r.close()
    assert src != src2
    first = _child(tmp_path, src)
    assert first["origin"] == "compiled" and first["n"] > 0
    entry = tmp_path / "cache" / f"{first['key']}.co"
    data = entry.read_bytes()
    assert data[:8] == b"WOJITCO1"
    (n,) = struct.unpack("<Q", data[8:16])
    assert n == first["n"] == len(data) - 48
    assert data[16:48] == hashlib.sha256(data[48:]).digest()  # the library's SHA-256 is FIPS 180-4's
    second = _child(tmp_path, src)
    assert second["origin"] == "disk" and second["key"] == first["key"] and second["n"] == first["n"]
    assert second["sec"] < 0.5
    other = _child(tmp_path, src2)
    assert other["origin"] == "compiled" and other["key"] != first["key"]
    flagged = _child(tmp_path, src, {"WOLOLO_JIT_FLAGS": "-DWO_LDS_NEXT_EAGER=1"})
    assert flagged["origin"] == "compiled" and flagged["key"] != first["key"]
    # a truncated / corrupted entry is not loaded
    entry.write_bytes(data[:-7] + b"garbage")
    again = _child(tmp_path, src)
    assert again["origin"] == "compiled" and again["key"] == first["key"]
    assert entry.read_bytes() == data  # rewritten, same object
    # off switch
    off = _child(tmp_path, src, {"WOLOLO_JIT_CACHE": "0"})
    assert off["origin"] == "compiled"
    # same process: the process cache.  (Its key may differ from the child's: the key
    # holds the loaded HIP runtime's version, and this process imported torch, whose
    # bundled HIP runtime / hiprtc / comgr then serve libwololo too -- another compiler.)
    monkeypatch.setenv("WOLOLO_JIT_CACHE", str(tmp_path / "cache"))
    n, origin, _, key = wl.jit_code_object(src, "gfx950")
    n2, origin2, _, key2 = wl.jit_code_object(src, "gfx950")
    assert origin2 == "process" and key2 == key and n2 == n


def test_jit_code_resources_from_the_kernel_descriptor(hostonly, monkeypatch):
    """wo_jit_code_resources: the specialised kernel's scratch bytes per lane and static
    LDS from its code object's AMDHSA kernel descriptor (what wo_renderer_kernel_info
    reports; no GPU).  csg32's kernel spills nothing; its LDS is the generator's."""
    r = wl.Renderer("res", max_nodes=4096)
    scenes.build("csg32", r)
    r.set_tracer("auto")
    monkeypatch.setenv("WOLOLO_JIT_CACHE", "0")
    scratch, lds = wl.jit_code_resources(r.jit_source(), "gfx950:sramecc+:xnack-")
    assert scratch == 0 and 16 * 1024 < lds < 64 * 1024, (scratch, lds)
    with pytest.raises(wl.WololoError):
        wl.jit_code_resources("this is not HIP", "gfx950")
    r.close()


def test_jit_compiles_with_the_system_hiprtc_under_torch(hostonly, monkeypatch):
    """A process that imported torch first runs the library on torch's bundled ROCm
    (HIP runtime, hiprtc, comgr: 7.0 in this image), whose compiler spilled
    csg32_nested's kernel (2 VGPRs, 12 B per lane; 3 % slower).  The specialised
    kernels then compile in wo_jitc, a process linked to the system ROCm's hiprtc:
    no scratch, and a key of its own (so the two compilers' objects never mix)."""
    import torch  # noqa: F401  (as bench.py)
    r = wl.Renderer("nested-src", max_nodes=4096)
    scenes.build("csg32_nested", r)
    r.set_tracer("auto")
    src = r.jit_source()
    monkeypatch.setenv("WOLOLO_JIT_CACHE", "0")
    scratch, lds = wl.jit_code_resources(src, "gfx950:sramecc+:xnack-")
    assert scratch == 0 and lds > 0, (scratch, lds)
    r.close()


_RENDER_CHILD = r"""
import json, sys, time
sys.path.insert(0, {root!r})
from csgrenderer_amd import scenes
from csgrenderer_amd import wololo as wl
r = wl.Renderer("cache-child", max_nodes=4096)
info = scenes.build("csg256_balanced", r)
t0 = time.perf_counter()
img = r.render(info.params(width=64, height=36, spp=2))
origin, sec = r.jit_info()
print(json.dumps({{"origin": origin, "sec": sec, "wall": time.perf_counter() - t0, "sum": float(img.sum()),
                   "path": r.trace_path()}}))
"""


@pytest.mark.gpu
def test_second_process_renders_csg256_without_compiling(tmp_path):
    """csg256 compiles for seconds; a second process with the same cache loads the code
    object from disk (< 0.5 s) and renders the same image."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WOLOLO_JIT_CACHE=str(tmp_path / "cache"))
    env.pop("WOLOLO_JIT_FLAGS", None)
    runs = []
    for _ in range(2):
        out = subprocess.run([sys.executable, "-c", _RENDER_CHILD.format(root=root)], env=env, check=True,
                             capture_output=True, text=True, timeout=150).stdout
        runs.append(json.loads(out.strip().splitlines()[-1]))
    assert runs[0]["path"] == runs[1]["path"] == "jit"
    assert runs[0]["origin"] == "compiled"
    assert runs[1]["origin"] == "disk" and runs[1]["sec"] < 0.5, runs
    assert runs[1]["sum"] == runs[0]["sum"]
    print(runs)


def _chain_scene(r, n, ops, seed):
    """A left-deep chain over n spheres, its operators cycling through `ops`."""
    rng = np.random.default_rng(seed)
    acc = r.sphere(1.0)
    for i in range(1, n):
        s = r.sphere(float(rng.uniform(0.2, 0.6)))
        op = {"u": r.union, "d": r.difference, "i": r.intersection}[ops[i % len(ops)]]
        acc = op(wl.arg(acc), wl.arg(s, tuple(float(x) for x in rng.uniform(-1.0, 1.0, 3))))
    return acc


def _random_tree(r, n, seed):
    """A random binary tree over n spheres and half-spaces, random operators."""
    rng = np.random.default_rng(seed)
    items = []
    for _ in range(n):
        if rng.random() < 0.8:
            items.append(r.sphere(float(rng.uniform(0.2, 0.8))))
        else:
            items.append(r.halfspace(tuple(float(x) for x in rng.normal(size=3))))
    while len(items) > 1:
        i = int(rng.integers(0, len(items) - 1))
        a, b = items[i], items[i + 1]
        op = (r.union, r.difference, r.intersection)[int(rng.integers(0, 3))]
        items[i:i + 2] = [op(wl.arg(a), wl.arg(b, tuple(float(x) for x in rng.uniform(-1.0, 1.0, 3))))]
    return items[0]


def _program_value(prog, nrec, bits):
    """The root's membership for each row of `bits` (n x words, uint32): the
    postfix program evaluated directly (BOUND records change nothing)."""
    st = []
    pc = 0
    while pc < nrec:
        rec = prog[pc]
        if rec.op == wl.WO_OP_PRIM:
            st.append(((bits[:, rec.u1 // 32] >> np.uint32(rec.u1 % 32)) & np.uint32(1)).astype(bool))
            pc += 1 + rec.u0
            continue
        if rec.op != wl.WO_OP_BOUND:
            b, a = st.pop(), st.pop()
            st.append({wl.WO_OP_UNION: a | b, wl.WO_OP_INTER: a & b, wl.WO_OP_DIFF: a & ~b,
                       wl.WO_OP_RDIFF: b & ~a}[rec.op])
        pc += 1
    assert len(st) == 1
    return st[0]


def _build_case(r, case):
    if case.startswith("csg"):
        scenes.build(case, r)
    elif case.startswith("chain"):
        _chain_scene(r, {"chain_uud": 128, "chain_uid": 90, "chain_i": 40, "chain_d": 70}[case],
                     case.split("_")[1], seed=len(case))
    elif case.startswith("unionpairs"):
        _union_of_pairs(r, 100 if case == "unionpairs" else 30, seed=5)
    else:
        _random_tree(r, 60 if case == "random_a" else 150, seed=ord(case[-1]))


def _union_of_pairs(r, n, seed):
    """A balanced union of n pairs (a op b, op cycling u/d/i) -- csg256_balanced's shape."""
    rng = np.random.default_rng(seed)
    items = []
    for i in range(n):
        a, b = r.sphere(float(rng.uniform(0.3, 0.6))), r.sphere(float(rng.uniform(0.3, 0.6)))
        op = (r.union, r.difference, r.intersection)[i % 3]
        items.append(op(wl.arg(a), wl.arg(b, (0.2, 0.1, 0.0))))
    while len(items) > 1:
        items = [r.union(wl.arg(items[i]), wl.arg(items[i + 1], tuple(float(x) for x in rng.uniform(-2, 2, 3))))
                 if i + 1 < len(items) else items[i] for i in range(0, len(items), 2)]
    return items[0]


def _compile_sweep(tmp_path, src, nw, ncull, lut=1, hbits=1):
    """The generated evaluation and toggle blocks (and the union-count table, or the
    truth tables with WO_JIT_LUT=`lut`) as a host function: evaluate at the start
    membership, then apply toggles, writing the root after each."""
    import ctypes
    import subprocess

    body = src[src.index("// WO_EVAL_BEGIN"):src.index("// WO_EVAL_END")]
    toggle = src[src.index("// WO_TOGGLE_BEGIN"):src.index("// WO_TOGGLE_END")]
    table = ""
    m = re.search(r"struct __attribute__\(\(aligned\(16\)\)\) WoUTerm \{[^}]*\};", src)
    if m:
        t = re.search(r"__constant__ WoUTerm kUTerm\[\d+\] = \{.*?\};", src, re.S)
        table = (m.group(0) + "\n" + t.group(0).replace("__constant__", "static const") + "\n"
                 "#define WO_UTERM kUTerm\n")
        assert "ucnt" in toggle
    m = re.search(r"__constant__ uint32_t kLut\[\d+\] = \{.*?\};", src, re.S)
    if m:
        table += m.group(0).replace("__constant__", "static const") + "\n#define WO_LUT kLut\n"
    for name, macro in (("kHInfo", "WO_HINFO"), ("kHTab", "WO_HTAB")):
        m = re.search(r"__constant__ uint32_t " + name + r"\[\d+\] = \{.*?\};", src, re.S)
        if m:
            table += m.group(0).replace("__constant__", "static const") + f"\n#define {macro} {name}\n"
    # the levelled tables' words: the LDS form's code (wodev::LdsBits) on a host array
    table = f"#define WO_JIT_LUT {lut}\n#define WO_HBITS_LDS {hbits}\n" + table
    # the levelled tables' unit values persist from the evaluation into the toggles
    m = re.search(r"^(.*)// WO_STATE_DECL", src, re.M)
    state = m.group(1) + "\n" if m else ""
    root_after = "(ucnt != 0)" if "kUTerm" in table else "r" if "kHTab" in table else None
    c = tmp_path / f"ev{lut}{hbits}.cpp"
    c.write_text("#include <stddef.h>\n#include <stdint.h>\n" + table +
                 "extern \"C\" void run(const uint32_t* all, int n, const uint32_t* ords, int nev, uint32_t* out) {\n"
                 f"  for (int i = 0; i < n; ++i) {{\n    uint32_t bits[{nw}];\n"
                 f"    for (int k = 0; k < {nw}; ++k) bits[k] = all[(size_t)i * {nw} + k];\n"
                 f"    uint32_t cull[{ncull}] = {{0}};\n    int ucnt = 0; (void)ucnt; bool was = false; (void)was;\n    uint32_t r;\n" +
                 state + body +
                 "    out[(size_t)i * (nev + 1)] = r;\n"
                 "    for (int e = 0; e < nev; ++e) {\n"
                 "      const uint64_t key = (uint64_t)ords[(size_t)i * nev + e] << 12;\n" + toggle +
                 ("      out[(size_t)i * (nev + 1) + e + 1] = " + (root_after or "0") + ";\n") +
                 "    }\n  }\n}\n")
    so = tmp_path / f"ev{lut}{hbits}.so"
    subprocess.run(["g++", "-O1", "-shared", "-fPIC", "-o", str(so), str(c)], check=True)
    lib = ctypes.CDLL(str(so))
    return lib, root_after is not None


@pytest.mark.parametrize("case", ["csg32_nested", "csg256_balanced", "csg256_chain", "chain_uud", "chain_uid",
                                  "chain_d", "random_a", "random_b", "unionpairs", "csg360_nested"])
def test_generated_root_evaluation(hostonly, tmp_path, case):
    """The generated root evaluation of the event-list form (the scenes whose root is
    not a union of small terms: flattened literal sets; decision lists for chains; the
    incremental count of a union of >= 8 literal-set terms) compiled on the host is the
    program's value for random membership words of several densities and for every
    single primitive, and -- with the union count -- after each of a run of toggles
    (the sweep's events)."""
    import ctypes

    r = wl.Renderer("eval", max_nodes=4096)
    _build_case(r, case)
    prog, nrec, nprim = r.program()
    src = r.jit_source()
    r.close()
    assert "WO_EVAL_BEGIN" in src, case
    if case in ("csg256_chain", "chain_uud", "chain_d"):
        assert "decision list" in src  # left-deep unions / differences of spheres: one list
        assert wl.jit_compile_check(src, "gfx950") == ""  # and hiprtc takes it
    if case in ("csg256_balanced", "unionpairs"):
        assert "kUTerm" in src  # a union of >= 12 literal-set terms: the incremental count
        assert wl.jit_compile_check(src, "gfx950") == ""
    if case == "csg32_nested":
        assert "kLut" in src  # two subtrees of <= 12 primitives: the truth-table evaluation
        assert wl.jit_compile_check(src, "gfx950") == ""
    if case == "csg360_nested":
        assert "kHTab" in src  # 309 primitives: levels of truth tables, updated per event
    for lut in ((1, 0) if "kLut" in src else (1,)):
        # the levelled tables' membership words: the LDS form (wodev::LdsBits) and registers
        for hbits in ((1, 0) if "WO_HBITS_LDS" in src else (1,)):
            _check_generated_eval(tmp_path, src, prog, nrec, nprim, lut, hbits)


def _check_generated_eval(tmp_path, src, prog, nrec, nprim, lut, hbits=1):
    import ctypes

    nw = (nprim + 31) // 32
    ncull = max(1, len(re.findall(r"cull\[(\d+)\] = 0u;", src)))
    lib, counted = _compile_sweep(tmp_path, src, nw, ncull, lut, hbits)
    rng = np.random.default_rng(7)
    rows = [np.eye(nprim, dtype=np.uint8), np.zeros((1, nprim), dtype=np.uint8)]  # every primitive alone
    for p in (0.01, 0.03, 0.1, 0.3, 0.5):
        rows.append((rng.random((2000, nprim)) < p).astype(np.uint8))
    mem = np.concatenate(rows)
    nev = 12 if counted else 0
    ords = rng.integers(0, nprim, size=(len(mem), max(nev, 1)), dtype=np.uint32)
    # a third of the rows toggle primitives of one neighbourhood (events of one term and its neighbours)
    ords[::3] = (ords[::3, :1] + rng.integers(0, 3, size=(len(ords[::3]), ords.shape[1]))) % nprim

    def pack(m):
        bits = np.zeros((len(m), nw), dtype=np.uint32)
        for k in range(nprim):
            bits[:, k // 32] |= m[:, k].astype(np.uint32) << np.uint32(k % 32)
        return bits

    out = np.zeros((len(mem), nev + 1), dtype=np.uint32)
    lib.run(pack(mem).ctypes.data_as(ctypes.c_void_p), ctypes.c_int(len(mem)),
            np.ascontiguousarray(ords).ctypes.data_as(ctypes.c_void_p), ctypes.c_int(nev),
            out.ctypes.data_as(ctypes.c_void_p))
    cur = mem.copy()
    for e in range(nev + 1):
        if e:
            cur[np.arange(len(cur)), ords[:, e - 1]] ^= 1
        want = _program_value(prog, nrec, pack(cur))
        got = out[:, e].astype(bool)
        assert np.array_equal(got, want), (e, int(np.count_nonzero(got != want)))


def _f32(h):
    return float(np.array([int(h, 16)], dtype=np.uint32).view(np.float32)[0])


@pytest.mark.parametrize("case", ["csg256_chain", "random_a"])
def test_spatial_groups_enclose_their_primitives(hostonly, case):
    """Spatial collect (scene_jit.c gen_spatial): each wave-level group test's sphere
    (centre and R, R^2 as emitted) encloses the bounding sphere of every primitive the
    group skips when culled, so a culled group never hides a primitive a ray meets;
    and every primitive is collected exactly once per pass.  (The event-list form over
    <= 64 primitives or a deep tree; the term form's groups:
    test_spatial_groups_enclose_their_terms.)"""
    r = wl.Renderer("sp", max_nodes=4096)
    _build_case(r, case)
    prog, nrec, nprim = r.program()
    src = r.jit_source()
    r.close()
    # each primitive's bounding sphere: its smallest sphere member
    pc_of = {prog[i].u1: i for i in range(nrec) if prog[i].op == wl.WO_OP_PRIM}
    sph = {}
    for o, pc in pc_of.items():
        best = None
        for m in range(prog[pc].u0):
            L = prog[pc + 1 + m]
            if L.op == wl.WO_LEAF_SPHERE:
                rr = math.sqrt(L.f[3])
                if best is None or rr < best[3]:
                    best = (L.f[0], L.f[1], L.f[2], rr)
        if best:
            sph[o] = best
    lines = src.splitlines()
    first_pass = lines[:next(i for i, l in enumerate(lines) if "WO_MARK(\"collect_end\")" in l)]
    groups = 0
    for i, l in enumerate(first_pass):
        m = re.search(r"// group (\d+) \((\d+) primitives\)", l)
        if not m:
            continue
        groups += 1
        lits = re.findall(r"0x([0-9a-f]{8})", "\n".join(first_pass[i:i + 12]))
        r2, cx, cy, cz, rad = (_f32(x) for x in lits[:5])
        # the guarded body: from the `if (!(cull...)) {` after the test block to its closing brace
        j = next(k for k in range(i, len(first_pass)) if first_pass[k].strip().startswith("if (!(cull["))
        ind = len(first_pass[j]) - len(first_pass[j].lstrip())
        k = j + 1
        while not (first_pass[k].strip() == "}" and len(first_pass[k]) - len(first_pass[k].lstrip()) == ind):
            k += 1
        ords = [int(x) for x in re.findall(r"// primitive (\d+) ", "\n".join(first_pass[j:k]))]
        assert len(ords) == int(m.group(2))
        for o in ords:
            c = sph[o]
            need = math.dist(c[:3], (cx, cy, cz)) + c[3]
            assert need <= rad and need * need <= r2 * (1 + 1e-6), (case, m.group(1), o, need, rad)
    assert groups >= 1
    # every primitive once in the first pass and once in the re-collect pass
    ords_all = [int(x) for x in re.findall(r"// primitive (\d+) ", src)]
    assert sorted(ords_all) == sorted(list(range(nprim)) * 2)


def _tree_regions(prog, nrec):
    """Per CSG node (postfix order) its children, primitive ordinals, bounds box, a
    sphere around its geometry and its relevance box, restated independently of
    scene_jit.c's rtree_build: a primitive's box from its sphere members and axis
    half-spaces, its sphere its smallest sphere member; a union's box the hull and its
    sphere the enclosing sphere of its operands', an intersection's box the meet and
    its sphere the smaller operand's, a difference's its left operand's (RDIFF: the
    right); the relevance box the meet of the boxes of the operands gating the node
    (an intersection's other operand, a difference's left one for its right one)."""
    INF = math.inf
    nodes, st = [], []
    for pc in range(nrec):
        r = prog[pc]
        if r.op == wl.WO_OP_PRIM:
            lo, hi, sph = [-INF] * 3, [INF] * 3, None
            for m in range(r.u0):
                L = prog[pc + 1 + m]
                if L.op == wl.WO_LEAF_SPHERE:
                    rr = math.sqrt(L.f[3])
                    for a in range(3):
                        lo[a], hi[a] = max(lo[a], L.f[a] - rr), min(hi[a], L.f[a] + rr)
                    if sph is None or rr < sph[3]:
                        sph = (L.f[0], L.f[1], L.f[2], rr)
                elif L.op == wl.WO_LEAF_HALFSPACE and 1 <= L.u1 <= 3:
                    a = L.u1 - 1
                    if L.f[a] > 0:
                        hi[a] = min(hi[a], L.f[3])
                    else:
                        lo[a] = max(lo[a], -L.f[3])
            nodes.append({"op": 0, "ords": [r.u1], "box": (lo, hi), "sph": sph})
            st.append(len(nodes) - 1)
        elif r.op in (wl.WO_OP_UNION, wl.WO_OP_INTER, wl.WO_OP_DIFF, wl.WO_OP_RDIFF):
            b, a = st.pop(), st.pop()
            A, B = nodes[a], nodes[b]
            if r.op == wl.WO_OP_UNION:
                box = ([min(x, y) for x, y in zip(A["box"][0], B["box"][0])],
                       [max(x, y) for x, y in zip(A["box"][1], B["box"][1])])
                sph = None
                if A["sph"] and B["sph"]:
                    (ca, ra), (cb, rb) = (A["sph"][:3], A["sph"][3]), (B["sph"][:3], B["sph"][3])
                    d = math.dist(ca, cb)
                    if d + rb <= ra:
                        sph = A["sph"]
                    elif d + ra <= rb:
                        sph = B["sph"]
                    else:
                        R = 0.5 * (d + ra + rb)
                        sph = tuple(ca[k] + (cb[k] - ca[k]) / d * (R - ra) for k in range(3)) + (R,)
            elif r.op == wl.WO_OP_INTER:
                box = ([max(x, y) for x, y in zip(A["box"][0], B["box"][0])],
                       [min(x, y) for x, y in zip(A["box"][1], B["box"][1])])
                cand = [x for x in (A["sph"], B["sph"]) if x]
                sph = min(cand, key=lambda q: q[3]) if cand else None
            else:
                keep = A if r.op == wl.WO_OP_DIFF else B
                box, sph = keep["box"], keep["sph"]
            nodes.append({"op": r.op, "l": a, "r": b, "ords": A["ords"] + B["ords"], "box": box, "sph": sph})
            st.append(len(nodes) - 1)
    root = st[-1]
    rel = {root: ([-INF] * 3, [INF] * 3)}
    meet = lambda x, y: ([max(p, q) for p, q in zip(x[0], y[0])], [min(p, q) for p, q in zip(x[1], y[1])])
    for i in range(len(nodes) - 1, -1, -1):
        n = nodes[i]
        if n["op"] == 0:
            continue
        c = rel[i]
        gate_l = n["op"] in (wl.WO_OP_INTER, wl.WO_OP_RDIFF)
        gate_r = n["op"] in (wl.WO_OP_INTER, wl.WO_OP_DIFF)
        rel[n["l"]] = meet(c, nodes[n["r"]]["box"]) if gate_l else c
        rel[n["r"]] = meet(c, nodes[n["l"]]["box"]) if gate_r else c
    for i, n in enumerate(nodes):
        n["rel"] = rel[i]
    return nodes, root


@pytest.mark.parametrize("case", ["csg32_nested", "csg360_nested"])
def test_relevance_groups_enclose_their_subtrees(hostonly, case):
    """The tree collect of the truth-table forms (scene_jit.c gen_rtree): each wave-level
    relevance group's sphere (centre and R, R^2 as emitted) encloses a region that holds
    the subtree's geometry where it is relevant -- the subtree's own sphere, or every
    corner of the meet of its bounds and relevance box -- so a culled group only ever
    zeroes bits that cannot change the root; the groups nest as the tree does, every
    primitive is collected at most once per pass, in the same order in both, and a
    primitive is left out only where the meet of its bounds and relevance box is empty."""
    r = wl.Renderer("rg", max_nodes=4096)
    _build_case(r, case)
    prog, nrec, nprim = r.program()
    src = r.jit_source()
    r.close()
    nodes, root = _tree_regions(prog, nrec)
    lines = src.splitlines()
    end1 = next(i for i, l in enumerate(lines) if 'WO_MARK("collect_end")' in l)
    first_pass = lines[:end1]
    # the groups in the order the tree walk emits them: nodes with >= min primitives,
    # depth first; matched by their primitive lists
    groups = 0
    for i, l in enumerate(first_pass):
        m = re.search(r"// relevance group (\d+) \((\d+) primitives\)", l)
        if not m:
            continue
        groups += 1
        lits = re.findall(r"0x([0-9a-f]{8})", "\n".join(first_pass[i:i + 12]))
        r2, cx, cy, cz, rad = (_f32(x) for x in lits[:5])
        j = next(k for k in range(i, len(first_pass)) if first_pass[k].strip().startswith("if (!(cull["))
        ind = len(first_pass[j]) - len(first_pass[j].lstrip())
        k = j + 1
        while not (first_pass[k].strip() == "}" and len(first_pass[k]) - len(first_pass[k].lstrip()) == ind):
            k += 1
        ords = sorted(int(x) for x in re.findall(r"// primitive (\d+) ", "\n".join(first_pass[j:k])))
        # the node: the subtree with exactly m.group(2) primitives containing these ordinals
        cands = [n for n in nodes if n["op"] and len(n["ords"]) == int(m.group(2)) and set(ords) <= set(n["ords"])]
        assert cands, (case, m.group(1), ords)
        ok = False
        for n in cands:
            s_ok = n["sph"] is not None and \
                math.dist(n["sph"][:3], (cx, cy, cz)) + n["sph"][3] <= rad * (1 + 1e-5)
            lo = [max(p, q) for p, q in zip(n["box"][0], n["rel"][0])]
            hi = [min(p, q) for p, q in zip(n["box"][1], n["rel"][1])]
            b_ok = all(math.isfinite(v) for v in lo + hi) and all(
                math.dist((x, y, z), (cx, cy, cz)) <= rad * (1 + 1e-5)
                for x in (lo[0], hi[0]) for y in (lo[1], hi[1]) for z in (lo[2], hi[2]))
            ok = ok or s_ok or b_ok
        assert ok, (case, m.group(1), rad)
        assert rad * rad <= r2 * (1 + 1e-5)
    assert groups >= 2
    # every primitive at most once per pass, the same ones in the same order in both passes
    first = [int(x) for x in re.findall(r"// primitive (\d+) ", "\n".join(first_pass))]
    second = [int(x) for x in re.findall(r"// primitive (\d+) ", "\n".join(lines[end1:]))]
    # a re-collect copy per sweep form (the batch sweep's and the event loop's)
    ncopies = 2 if "#if WO_SWEEP_BATCH" in src else 1
    assert len(set(first)) == len(first) and first * ncopies == second
    # left out: exactly where the primitive's bounds meet its relevance box in nothing
    # (the generator's slack may keep a near-empty one; never drop a non-empty one)
    for n in nodes:
        if n["op"]:
            continue
        lo = [max(p, q) for p, q in zip(n["box"][0], n["rel"][0])]
        hi = [min(p, q) for p, q in zip(n["box"][1], n["rel"][1])]
        if n["ords"][0] not in first:
            assert any(a > b for a, b in zip(lo, hi)), (case, n["ords"][0])


@pytest.mark.parametrize("case", ["csg32", "unionpairs_s"])
def test_spatial_groups_enclose_their_terms(hostonly, case):
    """The term form (a root that is a union of <= 2-literal conjunctions over <= 64
    primitives) groups terms, each bounded by its smallest positive literal's smallest
    sphere member (a term lies inside each positive literal): every group test's
    sphere encloses those of the terms it skips when culled, and every primitive is in
    exactly one term, once per pass."""
    r = wl.Renderer("sp", max_nodes=4096)
    _build_case(r, case)
    prog, nrec, nprim = r.program()
    src = r.jit_source()
    r.close()
    assert "// term mode:" in src
    pc_of = {prog[i].u1: i for i in range(nrec) if prog[i].op == wl.WO_OP_PRIM}

    def sphere(o):
        pc, best = pc_of[o], None
        for m in range(prog[pc].u0):
            L = prog[pc + 1 + m]
            if L.op == wl.WO_LEAF_SPHERE:
                rr = math.sqrt(L.f[3])
                if best is None or rr < best[3]:
                    best = (L.f[0], L.f[1], L.f[2], rr)
        return best

    term_re = re.compile(r"// term: (NOT )?primitive (\d+)(?: AND (NOT )?primitive (\d+))?")

    def term_sphere(m):
        lits = [(m.group(2), not m.group(1))] + ([(m.group(4), not m.group(3))] if m.group(4) else [])
        cands = [sphere(int(o)) for o, pos in lits if pos]
        cands = [c for c in cands if c]
        return min(cands, key=lambda c: c[3]) if cands else None

    lines = src.splitlines()
    first_pass = lines[:next(i for i, l in enumerate(lines) if "WO_MARK(\"collect_end\")" in l)]
    groups = 0
    for i, l in enumerate(first_pass):
        m = re.search(r"// group (\d+) \((\d+) primitives\)", l)
        if not m:
            continue
        groups += 1
        lits = re.findall(r"0x([0-9a-f]{8})", "\n".join(first_pass[i:i + 12]))
        r2, cx, cy, cz, rad = (_f32(x) for x in lits[:5])
        j = next(k for k in range(i, len(first_pass)) if first_pass[k].strip().startswith("if (!(cull["))
        ind = len(first_pass[j]) - len(first_pass[j].lstrip())
        k = j + 1
        while not (first_pass[k].strip() == "}" and len(first_pass[k]) - len(first_pass[k].lstrip()) == ind):
            k += 1
        for tm in term_re.finditer("\n".join(first_pass[j:k])):
            c = term_sphere(tm)
            assert c is not None, "a grouped term has a bounded positive literal"
            need = math.dist(c[:3], (cx, cy, cz)) + c[3]
            assert need <= rad and need * need <= r2 * (1 + 1e-6), (case, m.group(1), tm.group(0), need, rad)
    assert groups >= 1
    ords = []
    for tm in term_re.finditer(src):
        ords += [int(tm.group(2))] + ([int(tm.group(4))] if tm.group(4) else [])
    assert sorted(ords) == sorted(list(range(nprim)) * 2)


_TERM_HARNESS = r"""
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>
#define __device__
#define __forceinline__ inline
#define WO_T_MIN (1.0e-3f)
namespace wodev {
constexpr uint64_t kEmptyKey = ~0ull;
constexpr float kInf = INFINITY;
struct Ivl { float a, b; uint32_t ma, mb; };
inline uint64_t event_key_lo(float t, uint32_t lo) {
    uint32_t u;
    memcpy(&u, &t, 4);
    return ((uint64_t)u << 32) | lo;
}
// the device's v_min_f64 on keys as doubles (IEEE minNum: a quiet NaN operand gives
// the other operand, bits unchanged)
#define WO_WIN_F64 1
inline uint64_t key_min(uint64_t a, uint64_t b) {
    double x, y;
    memcpy(&x, &a, 8);
    memcpy(&y, &b, 8);
    const double r = std::fmin(x, y);
    uint64_t u;
    memcpy(&u, &r, 8);
    return u;
}
@TERM@
}  // namespace wodev
using namespace wodev;

static uint64_t st = 88172645463325252ull;
static uint32_t rnd() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (uint32_t)st; }
static float pick(const std::vector<float>& pool) { return pool[rnd() % pool.size()]; }

struct Term { int n; uint32_t ord[2]; bool pos[2]; };

// the general algorithm: every primitive event in key order, the root re-evaluated
static bool sweep(const std::vector<Ivl>& iv, const std::vector<Term>& terms, uint64_t& key, bool& after_val) {
    const float tmin = WO_T_MIN;
    const size_t np = iv.size();
    std::vector<char> in(np);
    std::vector<uint64_t> ev;
    for (size_t p = 0; p < np; ++p) {
        const bool ne = !(iv[p].a > iv[p].b);
        in[p] = ne && iv[p].a <= tmin && iv[p].b > tmin;
        if (ne && iv[p].a > tmin) ev.push_back(event_key_lo(iv[p].a, (uint32_t)p << 12));
        if (ne && iv[p].b > tmin && iv[p].b < kInf) ev.push_back(event_key_lo(iv[p].b, ((uint32_t)p << 12) | 2048u));
    }
    std::sort(ev.begin(), ev.end());
    auto root = [&]() {
        for (const Term& t : terms) {
            bool v = true;
            for (int k = 0; k < t.n; ++k) v = v && (t.pos[k] ? in[t.ord[k]] != 0 : in[t.ord[k]] == 0);
            if (v) return true;
        }
        return false;
    };
    bool r = root();
    for (uint64_t e : ev) {
        in[((uint32_t)e) >> 12] ^= 1;
        const bool r2 = root();
        if (r2 != r) { key = e; after_val = r2; return true; }
    }
    return false;
}

// the term method, as the specialised kernel's term mode emits it
template <bool kFirst>
static void term_pass(const std::vector<Ivl>& iv, const std::vector<Term>& terms, uint64_t after, uint64_t& best,
                      uint32_t& cnt) {
    for (const Term& t : terms) {
        const uint32_t o0 = t.ord[0];
        const TermLit x = term_lit(iv[o0], term_ka(o0, t.pos[0]), term_kb(o0, t.pos[0]));
        if (t.n == 1) {
            if (kFirst) cnt += (t.pos[0] ? term_in0(x) : !term_in0(x)) ? 1u : 0u;
            term_cands1<kFirst>(x, after, best);
            continue;
        }
        if (t.pos[0] && !x.valid) continue;  // the wave-level skip, per lane
        const uint32_t o1 = t.ord[1];
        const TermLit y = term_lit(iv[o1], term_ka(o1, t.pos[1]), term_kb(o1, t.pos[1]));
        if (kFirst)
            cnt += ((t.pos[0] ? term_in0(x) : !term_in0(x)) & (t.pos[1] ? term_in0(y) : !term_in0(y))) ? 1u : 0u;
        // kYFirst: the other literal's ordinal is the smaller (the generator's constant)
        if (o1 < o0) {
            if (t.pos[1]) term_cands_of<true, kFirst, true>(x, y, after, best);
            else term_cands_of<false, kFirst, true>(x, y, after, best);
            if (t.pos[0]) term_cands_of<true, kFirst, false>(y, x, after, best);
            else term_cands_of<false, kFirst, false>(y, x, after, best);
        } else {
            if (t.pos[1]) term_cands_of<true, kFirst, false>(x, y, after, best);
            else term_cands_of<false, kFirst, false>(x, y, after, best);
            if (t.pos[0]) term_cands_of<true, kFirst, true>(y, x, after, best);
            else term_cands_of<false, kFirst, true>(y, x, after, best);
        }
    }
}

static bool term_method(const std::vector<Ivl>& iv, const std::vector<Term>& terms, uint64_t& key, bool& after_val) {
    uint64_t best = kBestNone;
    uint32_t cnt = 0;
    term_pass<true>(iv, terms, 0ull, best, cnt);
    if (best == kBestNone) return false;
    const bool root = cnt != 0u;
    for (;;) {
        cnt = term_rises(best) ? cnt + 1u : cnt - 1u;
        if ((cnt != 0u) != root) { key = term_event(best); after_val = cnt != 0u; return true; }
        const uint64_t after = best;
        best = kBestNone;
        uint32_t unused = 0;
        term_pass<false>(iv, terms, after, best, unused);
        if (best == kBestNone) return false;
    }
}

extern "C" long run(int rays, int* hits) {
    const std::vector<float> pool = {-INFINITY, -2.0f, -0.5f, 0.0f, 1.0e-3f, 0.25f, 0.5f, 0.5f, 1.0f, 1.5f, 2.0f,
                                     2.0f, 3.0f, 4.5f, INFINITY};
    long bad = 0;
    *hits = 0;
    for (int r = 0; r < rays; ++r) {
        const int nt = 1 + (int)(rnd() % 5);
        std::vector<Term> terms;
        std::vector<Ivl> iv;
        for (int i = 0; i < nt; ++i) {
            Term t;
            t.n = 1 + (int)(rnd() % 2);
            for (int k = 0; k < t.n; ++k) {
                t.ord[k] = (uint32_t)iv.size();
                t.pos[k] = (rnd() % 4) != 0;
                Ivl v;
                v.a = (rnd() % 3) ? pick(pool) : pick(pool) + 0.37f * (float)(rnd() % 7);
                v.b = (rnd() % 3) ? pick(pool) : pick(pool) + 0.29f * (float)(rnd() % 9);
                v.ma = v.mb = 0u;
                iv.push_back(v);
            }
            terms.push_back(t);
        }
        uint64_t k1 = 0, k2 = 0;
        bool v1 = false, v2 = false;
        const bool h1 = sweep(iv, terms, k1, v1), h2 = term_method(iv, terms, k2, v2);
        *hits += h1 ? 1 : 0;
        if (h1 != h2 || (h1 && (k1 != k2 || v1 != v2))) ++bad;
    }
    return bad;
}
"""


def test_term_transitions_match_the_sweep(tmp_path):
    """The term mode's transition rule (wo_device_common.h, between WO_TERM_BEGIN and
    WO_TERM_END), compiled on the host, against the general algorithm -- every
    primitive event in key order, the root re-evaluated -- on random unions of one- and
    two-literal terms with random polarities and intervals: empty ones, ones holding
    t_min, unbounded ends and tied times (the key order breaks them).  Same hit key and
    the same root after it, on every ray."""
    import ctypes
    import os
    import subprocess

    hdr = open(os.path.join(os.path.dirname(__file__), "..", "csgrenderer_amd", "csrc", "wo_device_common.h")).read()
    term = hdr[hdr.index("// WO_TERM_BEGIN"):hdr.index("// WO_TERM_END")]
    c = tmp_path / "terms.cpp"
    c.write_text(_TERM_HARNESS.replace("@TERM@", term))
    so = tmp_path / "terms.so"
    subprocess.run(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-o", str(so), str(c)], check=True)
    lib = ctypes.CDLL(str(so))
    lib.run.restype = ctypes.c_long
    hits = ctypes.c_int(0)
    bad = lib.run(200000, ctypes.byref(hits))
    assert hits.value > 50000  # the cases hit often enough to mean something
    assert bad == 0, f"{bad} rays differ"


@pytest.mark.parametrize("case,want", [("csg360_nested", 1), ("csg256_chain", 0), ("csg256_balanced", 0),
                                       ("csg32_nested", 0), ("csg32", 0), ("csg512_balanced", 0)])
def test_levelled_tables_take_only_big_general_trees(hostonly, case, want):
    """The levelled truth tables (scene_jit.c hlut_plan) are generated for a general tree
    above lut_plan's 64 primitives whose levels of <= 8 units reach the root within 4
    (csg360_nested: 62, 10, 2, 1 units); a left-deep chain (too many levels: decision
    lists), a union of terms (the union count / term mode) and the small trees (one
    level of tables, or term mode) do not take them.  The renderer routes a general tree
    above WOLOLO_JIT_MAX_PRIMS to the specialised kernel exactly when they apply."""
    r = wl.Renderer("hl", max_nodes=4096)
    scenes.build(case, r)
    src = r.jit_source()
    r.close()
    assert f"#define WO_JIT_HLUT {want}\n" in src, case
    if want:
        m = re.search(r"// root by (\d+) levels of truth tables \(units per level:([\d ]+)\)", src)
        units = [int(x) for x in m.group(2).split()]
        assert int(m.group(1)) == len(units) <= 4 and units[-1] == 1
        assert all(a > b for a, b in zip(units, units[1:]))
        info = re.search(r"kHInfo\[(\d+)\]", src)
        assert int(info.group(1)) == 309 + sum(units[:-1])  # an entry per lower index per level


def _prim_bits(prog, nrec, P):
    """Membership of every primitive at points P (n, 3), float64 from the fp32 records,
    as words of bits (n x words, uint32) for _program_value."""
    P = np.asarray(P, dtype=np.float64)
    nprim = sum(1 for i in range(nrec) if prog[i].op == wl.WO_OP_PRIM)
    bits = np.zeros((len(P), (nprim + 31) // 32), dtype=np.uint32)
    pc = 0
    while pc < nrec:
        rec = prog[pc]
        if rec.op != wl.WO_OP_PRIM:
            pc += 1
            continue
        v = np.ones(len(P), dtype=bool)
        for m in range(rec.u0):
            L = prog[pc + 1 + m]
            f = np.array(L.f[:4], dtype=np.float64)
            v &= (((P - f[:3]) ** 2).sum(axis=1) <= f[3]) if L.op == wl.WO_LEAF_SPHERE else (P @ f[:3] <= f[3])
        bits[:, rec.u1 // 32] |= v.astype(np.uint32) << np.uint32(rec.u1 % 32)
        pc += 1 + rec.u0
    return bits


@pytest.mark.parametrize("case", ["csg32_nested", "csg360_nested"])
def test_recollect_behind_skip_keeps_the_root(hostonly, case):
    """the re-collect pass (WO_RECOLLECT_BEHIND) skips a relevance group whose
    sphere ends, on every lane, before the last processed key's t.  The skip is exact
    because a ray that has left a sphere never re-enters it (a sphere is convex) and,
    outside the group's sphere, the group's subtree is empty or gated off -- the first
    pass's cull argument, which holds for half-spaces and for a sphere drawn around the
    meet of the subtree's bounds with its relevance box alike.  Restated here: along
    random unit rays, with the skipped groups' primitives frozen at their membership
    at t_after (what the kernel's bits hold then), the root equals the true root at
    every sampled t > t_after.  Group spheres and margins are read from the emitted
    re-collect pass; membership in float64 from the fp32 records."""
    r = wl.Renderer("rb", max_nodes=4096)
    _build_case(r, case)
    prog, nrec, nprim = r.program()
    src = r.jit_source()
    r.close()
    lines = src.splitlines()
    end1 = next(i for i, l in enumerate(lines) if 'WO_MARK("collect_end")' in l)
    second = lines[end1:]
    groups = []  # (centre, margin literal, ordinals inside)
    for i, l in enumerate(second):
        if l.strip() != "#if WO_RECOLLECT_BEHIND":
            continue
        lits = re.findall(r"0x([0-9a-f]{8})", "\n".join(second[i + 1:i + 7]))
        c = np.array([_f32(x) for x in lits[:3]], dtype=np.float64)
        marg = _f32(lits[3])
        j = next(k for k in range(i, len(second)) if second[k].strip() == "#endif") + 1
        assert second[j].strip() == "{"
        ind = len(second[j]) - len(second[j].lstrip())
        k = j + 1
        while not (second[k].strip() == "}" and len(second[k]) - len(second[k].lstrip()) == ind):
            k += 1
        ords = [int(x) for x in re.findall(r"// primitive (\d+) ", "\n".join(second[j:k]))]
        groups.append((c, marg, ords))
    assert len(groups) >= 2, case
    rng = np.random.default_rng(11)
    lo = np.array([-6.0, -2.0, -6.0])
    hi = np.array([6.0, 6.0, 6.0])
    nray, nt = 600, 160
    skipped_any = 0
    for _ in range(nray):
        o = rng.uniform(lo, hi)
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        ta = float(rng.uniform(0.01, 12.0))
        skip = set()
        for c, marg, ords in groups:
            tca = float((c - o) @ d)
            if tca + 1e-4 * abs(tca) + marg < ta:
                skip.update(ords)
        if not skip:
            continue
        skipped_any += 1
        ts = ta + np.sort(rng.uniform(0.0, 30.0, nt))
        P = o[None, :] + ts[:, None] * d[None, :]
        true_bits = _prim_bits(prog, nrec, P)
        frozen0 = _prim_bits(prog, nrec, (o + ta * d)[None, :])[0]
        mask = np.zeros(true_bits.shape[1], dtype=np.uint32)
        for p in skip:
            mask[p // 32] |= np.uint32(1) << np.uint32(p % 32)
        frozen = (true_bits & ~mask) | (frozen0 & mask)
        assert np.array_equal(_program_value(prog, nrec, true_bits), _program_value(prog, nrec, frozen)), \
            (case, o, d, ta, sorted(skip))
    assert skipped_any >= nray // 10, (case, skipped_any)
