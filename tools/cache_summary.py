#!/usr/bin/env python3
"""Summarise tools/cache_profile.sh passes (gpurun_out/cache_<tag>/): per launch of
the path kernel, the L2 hit rate, the vector L1 hit rate (1 - L1-to-L2 read
requests / cache accesses), the mean L1-miss latency, LDS bank-conflict cycles per
LDS instruction and the instruction-cache hit rate.

    python tools/cache_summary.py gpurun_out/cache_rtiow [--copy r06_rtiow]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import counters  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--copy", default=None, help="write profiles/<prefix>_cache.json")
    a = ap.parse_args()
    c = {}
    for name in ("c1", "c2", "c3"):
        _, v = counters(a.dir, name)
        c.update(v)
    res = {"counters": c}
    g = c.get
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
        res["l2_hit_rate"] = g("TCC_HIT_sum") / max(g("TCC_HIT_sum") + g("TCC_MISS_sum"), 1.0)
    if g("TCP_TOTAL_CACHE_ACCESSES_sum"):
        res["l1_hit_rate"] = 1.0 - g("TCP_TCC_READ_REQ_sum", 0.0) / g("TCP_TOTAL_CACHE_ACCESSES_sum")
    if g("TCP_TCC_READ_REQ_sum"):
        res["l1_miss_latency_cycles"] = g("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / g("TCP_TCC_READ_REQ_sum")
    if g("SQ_INSTS_LDS"):
        res["lds_conflict_cycles_per_inst"] = g("SQ_LDS_BANK_CONFLICT", 0.0) / g("SQ_INSTS_LDS")
    if g("SQC_ICACHE_HITS") is not None and g("SQC_ICACHE_MISSES") is not None:
        res["icache_hit_rate"] = g("SQC_ICACHE_HITS") / max(g("SQC_ICACHE_HITS") + g("SQC_ICACHE_MISSES"), 1.0)
    json.dump(res, sys.stdout, indent=1)
    print()
    if a.copy:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        json.dump(res, open(os.path.join(root, "profiles", f"{a.copy}_cache.json"), "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
