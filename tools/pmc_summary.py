#!/usr/bin/env python3
"""Summarise a tools/profile_session.sh run (gpurun_out/prof_<tag>/): kernel
duration, HBM bytes per launch, instruction mix, lane utilisation and where the
wave cycles go, for the path-tracer kernel.  Optionally records the traffic in
profiles/pmc_traffic.json (key scene:WxH:spp:ranks:path) and copies the CSVs
under profiles/ with a round prefix.

    python tools/pmc_summary.py gpurun_out/prof_csg32_jit --key csg32:1920x1080:64:1:jit \\
        --save profiles/pmc_traffic.json --copy r02_csg32_jit
"""
import argparse
import csv
import glob
import json
import os
import shutil
import sys

KERNELS = ("wo_jit_pathtrace", "pathtrace_lanes_kernel", "pathtrace_kernel")


def _rows(d, pattern):
    files = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    out = []
    for f in files:
        out += list(csv.DictReader(open(f)))
    return files, out


def counters(d, name):
    files, rows = _rows(os.path.join(d, name), "*counter_collection.csv")
    per = {}
    for r in rows:
        if not any(k in r["Kernel_Name"] for k in KERNELS):
            continue
        per.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return files, {k: sum(v.values()) / len(v) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--key", default=None)
    ap.add_argument("--save", default=None)
    ap.add_argument("--copy", default=None, help="copy CSVs to profiles/<prefix>_*.csv")
    ap.add_argument("--timed", type=int, default=None,
                    help="also average the last N dispatches of the kernel trace (the bench's timed frames: "
                         "the first launches run at a ramping clock)")
    a = ap.parse_args()
    res = {}
    kfiles, krows = _rows(os.path.join(a.dir, "kstats"), "*kernel_stats.csv")
    for r in krows:
        if any(k in r["Name"] for k in KERNELS):
            res["kernel"] = r["Name"]
            res["calls"] = int(r["Calls"])
            res["avg_ms"] = float(r["AverageNs"]) / 1e6
    tfiles, trows = _rows(os.path.join(a.dir, "kstats"), "*kernel_trace.csv")
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trows
            if any(k in r["Kernel_Name"] for k in KERNELS)]
    if durs:
        res["median_ms"] = sorted(durs)[len(durs) // 2]
        if a.timed and len(durs) >= a.timed:
            res["timed_dispatches"] = a.timed
            res["timed_avg_ms"] = sum(durs[-a.timed:]) / a.timed
    # which code object each pass ran: the bench line's roofline.kernel_object (key,
    # scratch bytes per lane, VGPRs) from every pass's log; the passes must agree, and
    # the kernel trace's Scratch_Size is recorded beside it
    objs = {}
    for name in ("kstats", "fetch", "write", "pmc1", "pmc2"):
        lg = os.path.join(a.dir, name + ".log")
        if not os.path.exists(lg):
            continue
        for line in open(lg, errors="replace"):
            line = line.strip()
            if line.startswith("{") and '"roofline"' in line:
                try:
                    objs[name] = json.loads(line)["roofline"].get("kernel_object")
                except ValueError:
                    pass
    keys = {json.dumps(v, sort_keys=True) for v in objs.values()}
    res["kernel_object"] = next(iter(objs.values()), None)
    res["kernel_object_passes"] = sorted(objs)
    res["kernel_object_consistent"] = len(keys) == 1
    scr = sorted({r["Scratch_Size"] for r in trows if any(k in r["Kernel_Name"] for k in KERNELS)})
    res["trace_scratch_size"] = [int(x) for x in scr]
    ffiles, f = counters(a.dir, "fetch")
    wfiles, w = counters(a.dir, "write")
    p1files, p1 = counters(a.dir, "pmc1")
    p2files, p2 = counters(a.dir, "pmc2")
    if "FETCH_SIZE" in f and "WRITE_SIZE" in w:
        # KiB; FETCH_SIZE doubled (MI355X_MICROARCH.md: gfx950 tallies 128-B reads at 64 B)
        res["fetch_bytes"] = f["FETCH_SIZE"] * 2 * 1024
        res["write_bytes"] = w["WRITE_SIZE"] * 1024
        res["traffic_bytes"] = int(round(res["fetch_bytes"] + res["write_bytes"]))
    c = {**p1, **p2}
    res["counters"] = c
    if c.get("SQ_ACTIVE_INST_VALU"):
        res["lane_util_valu"] = c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64)
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        res["frac_wave_cycles"] = {k: c[k] / wc for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")
                                   if k in c}
    if c.get("GRBM_GUI_ACTIVE") and res.get("avg_ms"):
        res["clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / (res["avg_ms"] * 1e-3) / 1e9
    json.dump(res, sys.stdout, indent=1)
    print()
    if not res["kernel_object_consistent"]:
        print("ERROR: the passes ran different code objects: " + json.dumps(objs), file=sys.stderr)
        return 2
    if a.save and a.key and "traffic_bytes" in res:
        j = json.load(open(a.save)) if os.path.exists(a.save) else {}
        ko = res.get("kernel_object") or {}
        j[a.key] = {"bytes": res["traffic_bytes"], "kernel_key": ko.get("key"),
                    "scratch_bytes": ko.get("scratch_bytes")}
        json.dump(j, open(a.save, "w"), indent=1)
        print(f"recorded {a.key} = {res['traffic_bytes']} in {a.save}")
    if a.copy:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        for tag, files in (("kernel_stats", kfiles), ("kernel_trace", tfiles), ("pmc_fetch", ffiles), ("pmc_write", wfiles),
                           ("pmc_pmc1", p1files), ("pmc_pmc2", p2files)):
            for i, fn in enumerate(files[:1]):
                shutil.copy(fn, os.path.join(root, "profiles", f"{a.copy}_{tag}.csv"))
        json.dump(res, open(os.path.join(root, "profiles", f"{a.copy}_summary.json"), "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
