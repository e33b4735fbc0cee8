#!/usr/bin/env python3
"""Roofline line of k_vol_sched (config 4 volpath) from one profile directory.

Inputs (written by tools/profile_volsched.sh on the GPU box):
  <dir>/lookups.err  -- `MH_LOOKUPS k_vol_sched samples N lookups L` lines of the
                        MH_EXP_LOOKUPS diagnostic build (device-counted density-grid
                        lookups per launch; results are bit-identical to the release
                        build, so the count is the release kernel's too)
  <dir>/pmc.json     -- tools/make_pmc.py over the release build's rocprofv3 passes
                        (average launch duration, calibrated FETCH x2 + WRITE bytes)

Algorithmic bytes per launch = L x 32 B (the 8 float taps of a trilinear lookup)
+ N x 20 B (one R G B A W sample record), the figure of DESIGN.md section 3.
"""
import json
import os
import re
import sys

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E ~8 TB/s


def main(d):
    lines = [ln for ln in open(os.path.join(d, "lookups.err")) if ln.startswith("MH_LOOKUPS")]
    if not lines:
        sys.exit("no MH_LOOKUPS line (was the diagnostic library loaded?)")
    m = re.search(r"samples (\d+) lookups (\d+)", lines[-1])
    n, lookups = int(m.group(1)), int(m.group(2))
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
