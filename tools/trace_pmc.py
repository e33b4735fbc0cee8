#!/usr/bin/env python3
"""Summary of a tools/profile_trace.sh run: per stream-engine kernel
(k_wf_trace / k_wf_shadow) the launch time and the counters that say where a
traversal step waits.  usage: trace_pmc.py <dir>"""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").replace("mh::", "")[:40]


def load(d, prefix):
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    seen = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, prefix + "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Dispatch_Id"] not in seen[k]:
                seen[k].add(r["Dispatch_Id"])
                dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return ctr, dur


def main():
    d = sys.argv[1]
    sq, sqd = load(d, "sq")
    ta, _ = load(d, "ta")
    tl, _ = load(d, "tlb")
    bench = [json.loads(l) for l in open(os.path.join(d, "bench.txt")) if l.startswith("{")]
    if bench:
        print("bench:", json.dumps({k: bench[-1][k] for k in ("triangles", "msamples_s", "trace_grays_s", "rays_closest", "rays_shadow")}))
    for k in sorted(sq):
        if not (k.startswith("k_wf_trace") or k.startswith("k_wf_shadow")):
            continue
        s, a, t = sq[k], ta[k], tl[k]
        clk = s["GRBM_GUI_ACTIVE"] / 8 / sqd[k] if sqd[k] else 0
        cyc = sqd[k] * clk
        out = {
            "kernel": k, "ms_sum": round(sqd[k] * 1e3, 3), "clock_ghz": round(clk / 1e9, 3),
            "wait_any": round(s["SQ_WAIT_ANY"] / s["SQ_WAVE_CYCLES"], 3) if s["SQ_WAVE_CYCLES"] else None,
            "vmem_latency_cyc": round(s["SQ_INST_LEVEL_VMEM"] / s["SQ_INSTS_VMEM"], 1) if s["SQ_INSTS_VMEM"] else None,
            "valu_per_vmem": round(s["SQ_INSTS_VALU"] / s["SQ_INSTS_VMEM"], 1) if s["SQ_INSTS_VMEM"] else None,
            "vmem_rd_insts": s["SQ_INSTS_VMEM_RD"],
            "ta_busy_frac": round(a["TA_TA_BUSY_sum"] / (256 * cyc), 3) if cyc else None,
            "ta_stalled_by_tc_frac": round(a["TA_ADDR_STALLED_BY_TC_CYCLES_sum"] / (256 * cyc), 3) if cyc else None,
            "td_busy_frac": round(a["TD_TD_BUSY_sum"] / (256 * cyc), 3) if cyc else None,
            "l1_to_l2_latency_cyc": round(a["TCP_TCC_READ_REQ_LATENCY_sum"] / a["TCP_TCC_READ_REQ_sum"], 1) if a["TCP_TCC_READ_REQ_sum"] else None,
            "l1_accesses_per_vmem_rd": round(a["TCP_TOTAL_CACHE_ACCESSES_sum"] / s["SQ_INSTS_VMEM_RD"], 1) if s["SQ_INSTS_VMEM_RD"] else None,
            "l1_l2_reads_per_access": round(a["TCP_TCC_READ_REQ_sum"] / a["TCP_TOTAL_CACHE_ACCESSES_sum"], 3) if a["TCP_TOTAL_CACHE_ACCESSES_sum"] else None,
            "tlb_miss_frac": round(t["TCP_UTCL1_TRANSLATION_MISS_sum"] / max(1, t["TCP_UTCL1_TRANSLATION_MISS_sum"] + t["TCP_UTCL1_TRANSLATION_HIT_sum"]), 4),
            "l2_hit": round(t["TCC_HIT_sum"] / max(1, t["TCC_HIT_sum"] + t["TCC_MISS_sum"]), 3),
        }
        print(json.dumps(out))


if __name__ == "__main__":
    main()
