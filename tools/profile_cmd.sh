#!/bin/bash
# SQ / cache / traffic counter passes (separate --pmc passes, kernel-trace only)
# over an arbitrary python script.  usage: tools/profile_cmd.sh <outdir> <script.py> [args...]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-gpurun_out/pc}; shift
SCRIPT=$(cd "$(dirname "$1")" && pwd)/$(basename "$1"); shift
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
run() { timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT" -- python3 "$SCRIPT" $ARGS >> "$OUT/log.txt" 2>&1; }
ARGS="$*"
run --kernel-trace -o trace || exit 1
run --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -o sq_a || exit 1
run --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -o sq_b || exit 1
run --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -o tcc || exit 1
run --kernel-trace --pmc FETCH_SIZE -o fetch || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
d = sys.argv[1]
ctr = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "trace_kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mh::", "")[:40]
        dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mh::", "")[:40]
        ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(dur, key=lambda x: -sum(dur[x]))[:8]:
    c = ctr[k]; wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    hit = c.get("TCC_HIT_sum", 0); miss = c.get("TCC_MISS_sum", 0)
    lane = c.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * c.get("SQ_ACTIVE_INST_VALU", 1) or 1)
    print(f"{k:40s} ms={sum(dur[k])/1e6:8.2f} wait_any={c.get('SQ_WAIT_ANY',0)/wc:.2f} "
          f"wait_inst={c.get('SQ_WAIT_INST_ANY',0)/wc:.2f} active={c.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} "
          f"valu={c.get('SQ_ACTIVE_INST_VALU',0)/wc:.2f} lane={lane:.2f} vmem_rd={c.get('SQ_INSTS_VMEM_RD',0):.3e} "
          f"salu={c.get('SQ_INSTS_SALU',0):.3e} l2hit={hit/(hit+miss+1e-9):.3f} fetchMB={2*c.get('FETCH_SIZE',0)/1024:.1f}")
PY
