#!/usr/bin/env python3
"""Summary of tools/profile_pvb_traffic.sh: per variant, the prbvolpath
backward (k_vol_sched<PvBwdMachine>) and forward per-launch HBM bytes
(FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md,
calibrated at 2.000 / 1.000 in profiles/r3_prbvolpath_config4_pmc_summary.txt)
and the step time; the difference to `base` is the source's traffic."""
import collections
import csv
import glob
import json
import os
import sys


def per_launch(d, v, c):
    acc, ids = collections.defaultdict(float), collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, f"{v}_{c}*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mh::", "")
            if not k.startswith("k_vol_sched"):
                continue
            k = "bwd" if "PvBwd" in k else "fwd"
            acc[k] += float(r["Counter_Value"]) * 1024  # KiB -> B
            ids[k].add(r["Dispatch_Id"])
    return {k: acc[k] / len(ids[k]) for k in acc}


def main():
    d = sys.argv[1]
    rows = {}
    for v in ("base", "nomain", "nonee", "noatom"):
        f, w = per_launch(d, v, "FETCH_SIZE"), per_launch(d, v, "WRITE_SIZE")
        b = [json.loads(l) for l in open(os.path.join(d, f"bench_{v}.txt")) if l.startswith("{")]
        rows[v] = {"bwd_GB": round((2 * f.get("bwd", 0) + w.get("bwd", 0)) / 1e9, 2),
                   "bwd_fetch_GB": round(2 * f.get("bwd", 0) / 1e9, 2), "bwd_write_GB": round(w.get("bwd", 0) / 1e9, 2),
                   "fwd_GB": round((2 * f.get("fwd", 0) + w.get("fwd", 0)) / 1e9, 2),
                   "bench": b[-1] if b else None}
    base = rows["base"]["bwd_GB"]
    for v, r in rows.items():
        r["source_GB"] = round(base - r["bwd_GB"], 2) if v != "base" else None
        print(json.dumps({"variant": v, **r}))


if __name__ == "__main__":
    main()
