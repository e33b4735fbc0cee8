#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel trace + PMC passes) per kernel.

usage: pmc_summary.py <dir> [prefix ...]
Reports per kernel: calls, avg duration, VALU lane utilisation
(SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)), VALU/LDS/VMEM instruction
counts per call and HBM traffic per call.  HBM bytes follow MI355X_MICROARCH.md
§HBM: FETCH_SIZE (KiB) reads exactly half of a wide coalesced stream on gfx950
-> doubled; WRITE_SIZE (KiB) exact for 16-B streaming stores.
"""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    n = name.split("(")[0]
    for pre in ("void ", "mh::"):
        n = n.replace(pre, "")
    return n[:48]


def main():
    d = sys.argv[1]
    prefixes = sys.argv[2:] or None
    dur = collections.defaultdict(list)
    files = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    # durations from the plain --kernel-trace pass when present (PMC passes
    # serialise dispatches and inflate them)
    plain = [f for f in files if os.path.basename(f).startswith("trace")]
    for f in plain or files:
        if prefixes and not any(os.path.basename(f).startswith(p) for p in prefixes):
            continue
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        if prefixes and not any(os.path.basename(f).startswith(p) for p in prefixes):
            continue
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[(k, r["Counter_Name"])].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    out = {}
    print(f"{'kernel':48s} {'calls':>6s} {'avg_us':>10s} {'lane%':>6s} {'VALU/call':>11s} {'LDS/call':>10s} "
          f"{'VMEM/call':>10s} {'HBM_MB/call':>11s}")
    for k in sorted(dur, key=lambda x: -sum(dur[x])):
        c = ctr.get(k, {})
        ncall = len(dur[k])
        def per(name):
            n = len(calls.get((k, name), ())) or 1
            return c.get(name, 0.0) / n
        lane = (c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]) * 100
                if c.get("SQ_ACTIVE_INST_VALU") else float("nan"))
        hbm = (2 * per("FETCH_SIZE") + per("WRITE_SIZE")) * 1024 / 1e6 if ("FETCH_SIZE" in c or "WRITE_SIZE" in c) else float("nan")
        avg = sum(dur[k]) / ncall / 1e3
        print(f"{k:48s} {ncall:6d} {avg:10.1f} {lane:6.1f} {per('SQ_INSTS_VALU'):11.3e} {per('SQ_INSTS_LDS'):10.3e} "
              f"{per('SQ_INSTS_VMEM_RD') + per('SQ_INSTS_VMEM_WR'):10.3e} {hbm:11.2f}")
        out[k] = {"calls": ncall, "avg_us": avg, "lane_util_pct": lane, "hbm_bytes_per_call": hbm * 1e6,
                  "fetch_kib_per_call": per("FETCH_SIZE"), "write_kib_per_call": per("WRITE_SIZE")}
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
