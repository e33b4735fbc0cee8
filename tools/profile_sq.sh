#!/bin/bash
# SQ stall/issue counters (separate --pmc passes, kernel-trace only) for one
# forward bench step.  usage: tools/profile_sq.sh <outdir> [bench args...]
# SQ_PROG=<script relative to the repo> profiles that script instead (its
# arguments: the bench args, without bench.py's defaults)
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-gpurun_out/sq}; shift
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
PROG=${SQ_PROG:-bench.py}
if [ -n "$SQ_PROG" ]; then ARGS="$*"; else ARGS="--no-cpu --steps 1 --warmup 0 $*"; fi
run() { timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT" -- python3 "$ROOT/$PROG" $ARGS >> "$OUT/log.txt" 2>&1; }
run --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -o sq_a || exit 1
run --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS -o sq_b || exit 1
run --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -o sq_c || exit 1
run --kernel-trace --pmc SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM -o sq_d || exit 1
run --kernel-trace --pmc SQ_INSTS_SMEM SQ_IFETCH -o sq_e || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
d = sys.argv[1]
ctr = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mh::", "")[:40]
        ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(ctr.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k:40s} wave_cyc={wc:.3e} wait_any={c.get('SQ_WAIT_ANY',0)/wc:.2f} wait_inst={c.get('SQ_WAIT_INST_ANY',0)/wc:.2f} "
          f"active_any={c.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} valu={c.get('SQ_ACTIVE_INST_VALU',0)/wc:.2f} "
          f"lds={c.get('SQ_ACTIVE_INST_LDS',0)/wc:.2f} sca={c.get('SQ_ACTIVE_INST_SCA',0)/wc:.2f} "
          f"wait_lds={c.get('SQ_WAIT_INST_LDS',0)/wc:.2f} salu={c.get('SQ_INSTS_SALU',0):.3e} br={c.get('SQ_INSTS_BRANCH',0):.3e} "
          f"valu_i={c.get('SQ_INSTS_VALU',0):.3e} lds_i={c.get('SQ_INSTS_LDS',0):.3e} bankc={c.get('SQ_LDS_BANK_CONFLICT',0):.3e} "
          f"lane={c.get('SQ_THREAD_CYCLES_VALU',0)/(64*max(c.get('SQ_ACTIVE_INST_VALU',1),1)):.2f} "
          f"smem={c.get('SQ_INSTS_SMEM',0):.3e} ifetch={c.get('SQ_IFETCH',0):.3e} busy={c.get('SQ_BUSY_CYCLES',0):.3e}")
PY
