#!/usr/bin/env python3
"""profiles/pmc_traffic.json from a tools/profile_r2.sh run (summary.json):
per-kernel PMC HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, gfx950
corrections per MI355X_MICROARCH.md) and rocprof average duration.
usage: make_traffic.py <profile dir> <label>"""
import json
import os
import sys

d, label = sys.argv[1], sys.argv[2]
s = json.load(open(os.path.join(d, "summary.json")))
out = {"source": label, "kernels": {k: {"hbm_bytes_per_call": v["hbm_bytes_per_call"], "avg_us": v["avg_us"],
                                         "calls": v["calls"], "lane_util_pct": v["lane_util_pct"]}
                                     for k, v in s.items() if v["hbm_bytes_per_call"] == v["hbm_bytes_per_call"]}}
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
json.dump(out, open(os.path.join(root, "profiles", "pmc_traffic.json"), "w"), indent=1)
print(json.dumps(out["kernels"].get("k_wf_trace<true>")))
