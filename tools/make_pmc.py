#!/usr/bin/env python3
"""Per-kernel PMC summary of a tools/profile_r2.sh run -> <dir>/pmc.json.

HBM traffic: FETCH_SIZE / WRITE_SIZE (KiB) of each kernel, corrected by the
factors measured on tools/calib_fetch's known-byte kernels for the kernel's
access width (MI355X_MICROARCH.md: FETCH_SIZE under-reports 16-B/lane streams
by 2x on gfx950; other widths must be calibrated):
  k_wf_bounce*      path state as 16-B records (WfPacked)  -> 16-B factors
  k_wf_bounce_prb*  4-B SoA planes (WfState / WfPrb)       ->  4-B factors
VALU issue fraction: SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction on a
SIMD-32) / (1024 SIMDs x duration x clock), clock = GRBM_GUI_ACTIVE / 8 XCDs /
duration of the counter pass.  usage: make_pmc.py <dir>"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS = 1024
WIDTH = {"k_wf_bounce_prb": 4, "k_wf_bounce": 16}


def short(name):
    n = name.split("(")[0]
    for pre in ("void ", "mh::"):
        n = n.replace(pre, "")
    return n[:48]


def load(d, prefix):
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    seen = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, prefix + "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
            did = r.get("Dispatch_Id", "")
            if did not in seen[k]:
                seen[k].add(did)
                dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return ctr, {k: len(v) for k, v in seen.items()}, dur


def main():
    d = sys.argv[1]
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    sq, sq_calls, sq_dur = load(d, "sq")
    fe, fe_calls, _ = load(d, "fetch")
    wr, wr_calls, _ = load(d, "write")
    cf, cf_calls, _ = load(d, "calib_fetch")
    cw, cw_calls, _ = load(d, "calib_write")
    tc, tc_calls, _ = load(d, "tcc")  # optional pass: TCC_HIT_sum / TCC_MISS_sum
    known = 20 * (1 << 24) * 4  # tools/calib_fetch bytes per launch
    calib = {}
    for w in (4, 16):
        rk, wk = f"k_read{w}", f"k_write{w}"
        calib[w] = {"fetch": known / (cf[rk]["FETCH_SIZE"] * 1024 / cf_calls[rk]) if cf_calls.get(rk) else 2.0,
                    "write": known / (cw[wk]["WRITE_SIZE"] * 1024 / cw_calls[wk]) if cw_calls.get(wk) else 1.0}
    out = {"calibration": {str(k): v for k, v in calib.items()}, "kernels": {}}
    print("calibration (known bytes / counter bytes):", json.dumps(out["calibration"]))
    print(f"{'kernel':44s} {'calls':>5s} {'avg_us':>8s} {'GHz':>5s} {'valu_iss':>8s} {'wait_any':>8s} "
          f"{'wait_ins':>8s} {'HBM_MB':>8s} {'TB/s':>6s}")
    for k in sorted(dur, key=lambda x: -sum(dur[x])):
        n = len(dur[k])
        avg = sum(dur[k]) / n
        rec = {"calls": n, "avg_us": avg * 1e6}
        if sq_calls.get(k):
            c = sq[k]
            per = sq_calls[k]
            clk = c["GRBM_GUI_ACTIVE"] / 8 / sq_dur[k] if sq_dur[k] else 0.0
            rec["clock_ghz"] = clk / 1e9
            rec["valu_insts_per_call"] = c["SQ_INSTS_VALU"] / per
            rec["valu_issue_frac"] = (c["SQ_INSTS_VALU"] * 2) / (SIMDS * sq_dur[k] * clk) if clk else None
            wc = c["SQ_WAVE_CYCLES"] or 1
            rec["wait_any"] = c["SQ_WAIT_ANY"] / wc
            rec["wait_inst"] = c["SQ_WAIT_INST_ANY"] / wc
            rec["active_valu"] = c["SQ_ACTIVE_INST_VALU"] / wc
        fam = next((f for f in sorted(WIDTH, key=len, reverse=True) if k.startswith(f)), None)
        if fe_calls.get(k) and wr_calls.get(k):
            w = WIDTH.get(fam, 16)
            rb = fe[k]["FETCH_SIZE"] * 1024 / fe_calls[k]
            wb = wr[k]["WRITE_SIZE"] * 1024 / wr_calls[k]
            rec["fetch_bytes_raw"] = rb
            rec["write_bytes_raw"] = wb
            rec["access_width"] = w
            rec["hbm_bytes_per_call"] = rb * calib[w]["fetch"] + wb * calib[w]["write"]
        if tc_calls.get(k):
            h, m = tc[k].get("TCC_HIT_sum", 0.0), tc[k].get("TCC_MISS_sum", 0.0)
            rec["l2_hit"] = h / (h + m) if h + m else None
        out["kernels"][k] = rec
        hb = rec.get("hbm_bytes_per_call")
        print(f"{k:44s} {n:5d} {avg * 1e6:8.1f} {rec.get('clock_ghz', 0):5.2f} {rec.get('valu_issue_frac') or 0:8.3f} "
              f"{rec.get('wait_any', 0):8.2f} {rec.get('wait_inst', 0):8.2f} {(hb or 0) / 1e6:8.1f} "
              f"{(hb or 0) / avg / 1e12:6.2f}")
    json.dump(out, open(os.path.join(d, "pmc.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
