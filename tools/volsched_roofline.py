#!/usr/bin/env python3
"""Roofline line of k_vol_sched (config 4 volpath) from one profile directory.

Inputs (written by tools/profile_volsched.sh on the GPU box):
  <dir>/lookups.json -- bench.py --config 4's line: its roofline carries the release
                        kernel's device-counted density-grid lookups (mh_stats.grid_lookups)
  <dir>/pmc.json     -- tools/make_pmc.py over the release build's rocprofv3 passes
                        (average launch duration, calibrated FETCH x2 + WRITE bytes)

Algorithmic bytes per launch = L x 32 B (the 8 float taps of a trilinear lookup)
+ N x 20 B (one R G B A W sample record), the figure of DESIGN.md section 3.
"""
import json
import os
import sys

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E ~8 TB/s


def main(d):
    line = json.loads(open(os.path.join(d, "lookups.json")).read().strip().splitlines()[-1])
    rf = line["roofline"]
    n, lookups = int(rf["samples"]) // max(1, int(rf["launches_per_step"])), int(rf["grid_lookups"]) // max(1, int(rf["launches_per_step"]))
    pmc = json.load(open(os.path.join(d, "pmc.json")))["kernels"]
    name = next(k for k in pmc if k.startswith("k_vol_sched<VolMachine"))
    k = pmc[name]
    us = k["avg_us"]
    alg = lookups * 32 + n * 20
    achieved = alg / (us * 1e-6) / 1e9
    traffic = k.get("hbm_bytes_per_call")
    out = {
        "kernel": name, "samples": n, "lookups": lookups, "lookups_per_sample": round(lookups / n, 3),
        "algorithmic_bytes": alg, "avg_us": round(us, 1),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4),
                     "traffic": round(traffic) if traffic is not None else None},
        "traffic_over_algorithmic": round(traffic / alg, 2) if traffic else None,
        "valu_issue_frac": round(k.get("valu_issue_frac", 0.0), 3), "wait_any": round(k.get("wait_any", 0.0), 3),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_vs")
